// host_pathwriter.cpp — epp::PathWriter (src/PathWriter.cpp:7-112): plain host I/O.
#include <cstdlib>
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
    std::ostringstream os;
    for (const Vec3& p : pts) {
        for (int k = 0; k < 3; ++k) os << p[k] << " ";
        os << '\n';
    }
    std::ofstream f(file);
    if (!f.is_open()) {
        std::cerr << "Failed to open file for writing: " << file << std::endl;
        return;
    }
    const std::string text = os.str();
    f.write(text.data(), (std::streamsize)text.size());
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
    writePoints(folderPath + "/path_" + std::to_string(writeCount) + ".txt", path);
    ++writeCount;
}

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
