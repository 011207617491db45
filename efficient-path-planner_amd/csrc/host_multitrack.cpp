// host_multitrack.cpp — epp::planTracks (include/epp/MultiTrackPlanner.h): one host thread
// per GPU, each with its own OnlineTrajGenerator per track (its World, planner scratch and
// streams live on that GPU), then the waypoint sets all-gathered over RCCL in rounds of one
// set per rank.
#include <hip/hip_runtime_api.h>

#include <exception>
#include <string>
#include <memory>
#include <stdexcept>
#include <thread>

#include "epp.h"
#include "epp/MultiTrackPlanner.h"
#include "epp/OnlineTrajGenerator.h"
#include "host_scratch.h"

namespace epp {

std::vector<TrackResult> planTracks(const std::vector<TrackProblem>& tracks, const std::string& configPath,
                                    const std::vector<int>& devices, double takeoffTime) {
    const int n = (int)devices.size();
    if (n < 1) throw std::invalid_argument("planTracks: no devices");
    std::vector<TrackResult> out(tracks.size());
    std::vector<epp_comm*> comms(n, nullptr);
    check(epp_comm_init_all(n, devices.data(), comms.data()), "planTracks: RCCL communicators");
    struct Release {
        std::vector<epp_comm*>& c;
        ~Release() {
            for (epp_comm* x : c) epp_comm_destroy(x);
        }
    } release{comms};
    const int rounds = (int)((tracks.size() + n - 1) / n);
    constexpr int32_t kCap = 4096;  // waypoints per track
    std::vector<std::vector<double>> gathered(n, std::vector<double>((size_t)n * kCap * 3));
    std::vector<std::vector<int32_t>> counts(n, std::vector<int32_t>(n));
    // Error protocol: a rank whose plan throws still takes part in the round's exchange,
    // with count -1; every rank then gets EPP_ERR_PEER from the same all-gather and leaves
    // the loop at the same round, so no rank is left waiting in RCCL.  A rank whose exchange
    // itself fails past the counts aborts every communicator (epp_comm_abort: the others'
    // polled waits end with EPP_ERR_PEER), and every wait has a deadline (epp.h).  The caller gets the
    // exception of the lowest failed rank (its own message, e.g. "Path not found").  A
    // capacity error is reported identically on all ranks by the all-gather as well.
    std::vector<std::exception_ptr> err(n);
    std::vector<char> own(n, 0);  // err[r] is rank r's own failure (not a peer's)
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            if (hipSetDevice(devices[r]) != hipSuccess) {
                err[r] = std::make_exception_ptr(std::runtime_error("planTracks: hipSetDevice"));
                own[r] = 1;
            }
            for (int k = 0; k < rounds; ++k) {
                const size_t t = (size_t)k * n + r;
                std::vector<double> wp;
                if (!err[r] && t < tracks.size()) {
                    try {
                        const TrackProblem& p = tracks[t];
                        OnlineTrajGenerator otg(p.start, p.goal, p.gates, p.obstacles, configPath);
                        otg.preComputeTraj(takeoffTime);
                        out[t].trajectory = otg.getPlannedTraj();
                        out[t].device = devices[r];
                        for (const Vec3& v : otg.getWaypoints()) wp.insert(wp.end(), {v.x, v.y, v.z});
                    } catch (...) {
                        err[r] = std::current_exception();
                        own[r] = 1;
                    }
                }
                // every rank takes part in every round (a rank without a track sends none,
                // a failed rank sends -1)
                const int32_t cnt = err[r] ? -1 : (int32_t)(wp.size() / 3);
                const epp_status st = epp_comm_allgather_waypoints(comms[r], wp.data(), cnt, kCap, gathered[r].data(),
                                                                   counts[r].data());
                if (st != EPP_OK) {
                    if (!err[r])
                        err[r] = std::make_exception_ptr(std::runtime_error(std::string("planTracks: all-gather: ") +
                                                                            epp_last_error()));
                    // EPP_ERR_PEER / EPP_ERR_CAPACITY come from the counts every rank holds:
                    // every rank breaks at this round.  Any other failure is this rank's own
                    // (a HIP error, a timeout) and may have left the others inside the data
                    // all-gather: abort every communicator, so their waits return at once.
                    if (st != EPP_ERR_PEER && st != EPP_ERR_CAPACITY)
                        for (epp_comm* x : comms) (void)epp_comm_abort(x);
                    break;
                }
                if (r == 0)  // rank 0's copy fills the results (all ranks hold the same)
                    for (int q = 0; q < n; ++q) {
                        const size_t tq = (size_t)k * n + q;
                        if (tq >= tracks.size()) continue;
                        const double* src = gathered[0].data() + (size_t)q * kCap * 3;
                        out[tq].waypoints.clear();
                        for (int i = 0; i < counts[0][q]; ++i)
                            out[tq].waypoints.emplace_back(src[3 * i], src[3 * i + 1], src[3 * i + 2]);
                    }
            }
        });
    for (auto& t : th) t.join();
    for (int r = 0; r < n; ++r)
        if (err[r] && own[r]) std::rethrow_exception(err[r]);
    for (const auto& e : err)
        if (e) std::rethrow_exception(e);
    return out;
}

}  // namespace epp
