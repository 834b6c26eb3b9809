// anx/v5.hpp — the device-resident multi-GPU runtime (the reference's planned V5, README.md:157-166:
// "pass device pointers to MPI ... remove staging"), shared by the `anx --version v5` CLI and the
// C ABI that bench.py / anx.parallel.workloads drive.
//
// One step over a hybrid batch x rows plan (anx/plan.hpp):
//   scatter   root X[images, tile.in rows] -> every rank's Tile             (transport, io stream)
//   stage1    conv1 + ReLU + pool1 into the conv2 window, chunk by chunk   (compute stream)
//   halo_p1   pool1 rows between row neighbours, one transfer list per chunk (halo stream), so the
//             halo of chunk c moves while stage1 computes chunk c+1 and stage2(c) waits only for it
//   stage2    conv2 + ReLU + pool2 + LRN of each chunk                      (compute stream)
//   gather    Y[images, tile.out rows] -> root YFull                        (transport, io stream)
// Steady state is pipelined across steps: scatter(k+1) and gather(k) run on the io stream while the
// compute stream runs step k; no stream is synchronised with the host inside a step. Weights reach
// every rank by an RCCL broadcast from the root's device (reference M4/M5 MPI_Bcast,
// v4_mpi_cuda/src/main_mpi_cuda.cpp:47-50).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "anx/comm.hpp"
#include "anx/engine.hpp"
#include "anx/plan.hpp"
#include "anx/schedule.hpp"

namespace anx {

struct V5Options {
  int batch = 1024;
  // row split inside each group of ranks: -1 = auto (balanced_row_ways), 0 = batch first, rows only
  // below one image per rank (make_hybrid_plan's auto), r > 0 = groups of r ranks (np = the
  // reference's pure row split)
  int row_ways = -1;
  Decomp mode = Decomp::PerLayer;
  std::string transport = "auto";  // auto | rccl | peer
  int chunks = 0;                  // halo pipeline chunks per step (0 = auto)
  int pipeline = -1;               // scatter(k+1) / gather(k) on the io stream: -1 auto, 0 off, 1 on
  bool poison = false;             // NaN-fill every consumed buffer after use (ordering tests)
  std::string peer_sync;           // peer transport ordering: "" (default) | flags | notes
  Impl impl = Impl::Mfma;
  Knobs knobs = default_knobs();
};

// Decomposition quality of a plan: output rows per rank (max / mean, 1.0 = balanced) and the conv1
// rows computed twice (anx/plan.hpp conv1_redundancy; 0 for a pure batch split).
struct PlanStats {
  int groups = 1, row_ways = 1;
  double rows_max = 0, rows_mean = 0, imbalance = 1, conv1_redundancy = 0, images_max = 0;
};
PlanStats plan_stats(const HybridPlan& p);

// Row ways a balanced default uses for `batch` images over `np` ranks: the fewest row ways r (r | np)
// whose per-rank work max / mean is within 1.1 (images split over np / r groups, 13 output rows over
// r ranks), which keeps the halo exchange of the row split without the 8-way split's imbalance
// (output rows 2,2,2,2,2,1,1,1: max / mean 1.23) and redundant Conv1. At least 2 when np > 1 so the
// V5 halo path runs; batch < np / r images fall back to finer row splits.
int balanced_row_ways(int np, int batch, int H = kInH, int W = kInW);

// V5 transport by node: auto = RCCL when every rank of this node has its own GPU or the job spans
// nodes, else peer (IPC, ranks share a GPU). Throws for a combination that cannot run.
std::string pick_v5_transport(const std::string& want, const RankInfo& ri, int ndev, bool dry);

// The plan, schedule and halo chunking of a V5 job: identical on every rank (a pure function of the
// job shape), which is what keeps every rank's sequence of transport calls the same.
struct V5Layout {
  HybridPlan plan;
  Schedule sched;
  int row_ways = 1, chunks = 1;
  std::vector<std::vector<Transfer>> halo_chunks;  // chunk_of(P1Halo list, c, chunks)
  // every transfer of one step in issue order: scatter, halo chunks, gather
  std::vector<Transfer> step_transfers() const;
};
V5Layout make_v5_layout(int np, const BlockSpec& b1, const BlockSpec& b2, int H, int W, const V5Options& o);

class V5Runtime {
 public:
  // Collective over `c`. Weights: the root's `w` is broadcast device-to-device by the transport (RCCL
  // broadcast / IPC copy); the other ranks' `w` is ignored.
  V5Runtime(HostComm& c, const RankInfo& ri, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
            const HostWeights& w, const V5Options& o);
  ~V5Runtime();
  V5Runtime(const V5Runtime&) = delete;
  V5Runtime& operator=(const V5Runtime&) = delete;

  // Collective: the root's `host_x` (the global batch [batch, H, W, C0]) becomes the input of every
  // following step (other ranks pass nullptr). Drains the pipeline first.
  void set_input(const float* host_x);
  // Enqueue one step (pipelined with its neighbours when the pipeline is on). No host sync.
  void step();
  // Wait for every enqueued step on every stream of this rank.
  void sync();
  // Root: the output of the last step [batch, Hp2, Wp2, C2] into host memory (syncs first).
  void output(float* host_y);
  // Mean ms per step since the last reset, by phase, on the compute stream's critical path:
  // scatter (waiting for the input), stage1, halo_p1 (waiting for halo chunks), stage2, gather
  // (end of stage2 to end of the gather). Syncs first.
  std::vector<std::pair<std::string, double>> phase_ms();
  void reset_phases();

  const V5Layout& layout() const { return lay_; }
  PlanStats stats() const { return plan_stats(lay_.plan); }
  const char* transport() const;
  bool pipelined() const { return pipeline_; }
  long steps() const;
  std::string describe_json() const;

 private:
  struct Impl_;
  std::unique_ptr<Impl_> p_;
  V5Layout lay_;
  bool pipeline_ = false;
};

// Record-only schedule of rank `rank` of `np` (no GPU, no communication): the transfers its transport
// would issue in one step, in issue order (--dry-run, tests).
std::vector<std::string> v5_dry_schedule(int rank, int np, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
                                         const V5Options& o, const std::string& transport);

}  // namespace anx
