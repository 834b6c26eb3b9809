// anx/v4.hpp — the host-staged multi-GPU runtime (the reference's V4, v4_mpi_cuda/src/main_mpi_cuda.cpp:
// 52-130: the batch lives in the root's host memory, input rows + halo go out, output rows come back),
// re-designed so that host staging is neither serial nor funnelled through one PCIe link:
//
//   * the batch and the output live in ONE shared host segment (POSIX shared memory, pinned in every
//     rank with hipHostRegister): each rank DMAs its own images x input rows (overlap tiles: the halo
//     rows included) straight from it over its own GPU's host link, and DMAs its output rows back into
//     it — there is no root H2D followed by a device scatter;
//   * a rank's share is cut into image chunks: H2D(c+1) on the h2d stream, tile_forward(c) on the
//     compute stream and D2H(c-1) on the d2h stream overlap; device buffers alternate by step parity,
//     so step k+1's copies overlap step k's tail too. No host synchronisation inside a step.
//
// Single node (the segment is node-local shared memory). Weights: host broadcast from the root (the
// reference's MPI_Bcast, main_mpi_cuda.cpp:47-50).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "anx/comm.hpp"
#include "anx/engine.hpp"
#include "anx/plan.hpp"

namespace anx {

struct V4Options {
  int batch = 256;
  int row_ways = -1;  // -1 the cost model's pick (anx/cost.hpp), 0 batch first, r > 0 groups of r ranks
  std::string cost;   // cost-model overrides for that pick ("name=value;...")
  int chunks = 0;     // image chunks per rank and step (0 = auto)
  Impl impl = Impl::Mfma;
  Knobs knobs = default_knobs();
};

class V4Runtime {
 public:
  // Collective over `c`. The root's `w` is broadcast over the host channel.
  V4Runtime(HostComm& c, const RankInfo& ri, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
            const HostWeights& w, const V4Options& o);
  ~V4Runtime();
  V4Runtime(const V4Runtime&) = delete;
  V4Runtime& operator=(const V4Runtime&) = delete;

  // The shared pinned segment, mapped in every rank: input [batch, H, W, C0] (write it, then call
  // input_ready()) and output [batch, Hp2, Wp2, C2] (complete after sync_all()).
  float* host_input() const;
  const float* host_output() const;
  // Collective: the input segment was (re)written by some rank; drains every rank's pipeline first.
  void input_ready();
  void step();     // enqueue one step, no host sync
  void sync();     // this rank's streams
  void sync_all();  // collective: every rank's streams (the output segment is complete)
  // Mean ms per step since the last reset: h2d (first to last H2D of the step on the h2d stream),
  // compute (first to last tile on the compute stream, waits included), d2h (end of compute to the
  // last D2H). Syncs first.
  std::vector<std::pair<std::string, double>> phase_ms();
  void reset_phases();
  // This rank's host link alone: GB/s of one H2D of its whole share in the step's copy pattern
  // (reps copies on the h2d stream, timed by events; the rate the H2D stage is bound by).
  double probe_h2d_gbps(int reps = 5);
  size_t h2d_bytes_per_step() const;  // this rank's
  size_t d2h_bytes_per_step() const;
  int chunks() const;
  const HybridPlan& plan() const;
  std::string describe_json() const;

 private:
  struct Impl_;
  std::unique_ptr<Impl_> p_;
};

}  // namespace anx
