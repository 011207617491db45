// epp/PathWriter.h — debug text dumps of OnlineTrajGenerator (the reference's
// include/PathWriter.h, src/PathWriter.cpp:7-112): path_<n>.txt per planned waypoint
// list, checkpoints.txt, and appended gates.txt / obstacles.txt lines, in the
// reference's stream formatting.  OnlineTrajGenerator writes to "path_segments" like the
// reference; EPP_PATH_WRITER=0 turns the dumps off.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "epp/types.h"

namespace epp {

class PathWriter {
public:
    // creates the folder, or removes the regular files already in it
    explicit PathWriter(const std::string& folderPath);
    void writePath(const std::vector<Vec3>& path);
    // The same write on the writer's own thread (started at the first call): returns at
    // once, so the caller's next step overlaps the file I/O; wait() returns when every such
    // write is on disk (OnlineTrajGenerator waits before its call returns, so the files
    // are there when the reference's would be).
    void writePathAsync(const std::vector<Vec3>& path);
    void wait();
    ~PathWriter();
    PathWriter(PathWriter&&) noexcept;
    PathWriter& operator=(PathWriter&&) noexcept;
    void updateGatePos(int gateId, const std::vector<double>& gateInfo);
    void updateObstaclePos(int obstacleId, const std::vector<double>& pose);
    void writeCheckpoints(const std::vector<Vec3>& checkpoints);
    bool enabled() const { return enabled_; }

private:
    std::string folderPath;
    int writeCount = 0;
    bool enabled_ = true;
    struct Worker;
    std::unique_ptr<Worker> worker_;
};

}  // namespace epp
