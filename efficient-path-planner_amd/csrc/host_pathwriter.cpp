// host_pathwriter.cpp — epp::PathWriter (src/PathWriter.cpp:7-112): plain host I/O.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>

#include "epp/PathWriter.h"

namespace epp {
namespace {

// Eigen's default `<< row.transpose()`: every coefficient right-aligned to the widest
// one (default stream precision), separated by one space
void writeEigenRow(std::ostream& os, const std::vector<double>& v) {
    size_t width = 0;
    for (double x : v) {
        std::ostringstream ss;
        ss.copyfmt(os);
        ss << x;
        width = std::max(width, ss.str().size());
    }
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) os << " ";
        os.width((std::streamsize)width);
        os << v[i];
    }
}

// (the reference flushes every line with std::endl; the same text is formatted in memory
// and written with one call: a path dump per plan cost ~40 us of syscalls)
void writePoints(const std::string& file, const std::vector<Vec3>& pts) {
    // "%.6g" is the default-stream formatting of a double (libstdc++ formats `os << x`
    // through the same printf conversion), so the text is the reference's; one write(2)
    // on a plain descriptor (an ofstream's construction and locale cost more than the text)
    std::string text;
    text.reserve(pts.size() * 40);
    char buf[64];
    for (const Vec3& p : pts) {
        for (int k = 0; k < 3; ++k) {
            const int n = std::snprintf(buf, sizeof(buf), "%.6g ", p[k]);
            text.append(buf, (size_t)std::max(n, 0));
        }
        text.push_back('\n');
    }
    const int fd = ::open(file.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) {
        std::cerr << "Failed to open file for writing: " << file << std::endl;
        return;
    }
    size_t off = 0;
    while (off < text.size()) {
        const ssize_t w = ::write(fd, text.data() + off, text.size() - off);
        if (w <= 0) break;
        off += (size_t)w;
    }
    ::close(fd);
}

void appendRow(const std::string& file, int id, const std::vector<double>& row) {
    std::ofstream f(file, std::ios_base::app);
    if (!f.is_open()) {
        std::cerr << "Failed to open file for writing: " << file << std::endl;
        return;
    }
    f << "id: " << id << " info: ";
    writeEigenRow(f, row);
    f << std::endl;
}

}  // namespace

PathWriter::PathWriter(const std::string& folder) : folderPath(folder) {
    const char* env = std::getenv("EPP_PATH_WRITER");
    enabled_ = !(env && std::string(env) == "0");
    if (!enabled_) return;
    namespace fs = std::filesystem;
    std::error_code ec;
    if (!fs::exists(folderPath, ec)) {
        fs::create_directories(folderPath, ec);
        std::cout << "Folder created: " << folderPath << std::endl;
    } else {
        for (const auto& e : fs::directory_iterator(folderPath, ec))
            if (e.is_regular_file(ec)) fs::remove(e.path(), ec);
    }
}

void PathWriter::writePath(const std::vector<Vec3>& path) {
    if (!enabled_) return;
    wait();  // (queued writes first: the files keep their order)
    writePoints(folderPath + "/path_" + std::to_string(writeCount) + ".txt", path);
    ++writeCount;
}

struct PathWriter::Worker {
    std::mutex mu;
    std::condition_variable cv, idle;
    std::deque<std::pair<std::string, std::vector<Vec3>>> q;
    int busy = 0;
    bool stop = false;
    std::thread t;
    Worker() {
        t = std::thread([this] {
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                cv.wait(lk, [this] { return stop || !q.empty(); });
                if (q.empty()) return;  // (stop, nothing left)
                auto job = std::move(q.front());
                q.pop_front();
                ++busy;
                lk.unlock();
                writePoints(job.first, job.second);
                lk.lock();
                --busy;
                if (q.empty() && busy == 0) idle.notify_all();
            }
        });
    }
    ~Worker() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        t.join();
    }
};

void PathWriter::writePathAsync(const std::vector<Vec3>& path) {
    if (!enabled_) return;
    if (!worker_) worker_ = std::make_unique<Worker>();
    {
        std::lock_guard<std::mutex> lk(worker_->mu);
        worker_->q.emplace_back(folderPath + "/path_" + std::to_string(writeCount) + ".txt", path);
    }
    worker_->cv.notify_one();
    ++writeCount;
}

void PathWriter::wait() {
    if (!worker_) return;
    std::unique_lock<std::mutex> lk(worker_->mu);
    worker_->idle.wait(lk, [this] { return worker_->q.empty() && worker_->busy == 0; });
}

PathWriter::~PathWriter() = default;  // (the worker's destructor finishes its queue)
PathWriter::PathWriter(PathWriter&&) noexcept = default;
PathWriter& PathWriter::operator=(PathWriter&&) noexcept = default;

void PathWriter::updateGatePos(int gateId, const std::vector<double>& gateInfo) {
    if (enabled_) appendRow(folderPath + "/gates.txt", gateId, gateInfo);
}

void PathWriter::updateObstaclePos(int obstacleId, const std::vector<double>& pose) {
    if (enabled_) appendRow(folderPath + "/obstacles.txt", obstacleId, pose);
}

void PathWriter::writeCheckpoints(const std::vector<Vec3>& checkpoints) {
    if (enabled_) writePoints(folderPath + "/checkpoints.txt", checkpoints);
}

}  // namespace epp
