// anx/v5.hpp — the device-resident multi-GPU runtime (the reference's planned V5, README.md:157-166:
// "pass device pointers to MPI ... remove staging"), shared by the `anx --version v5` CLI and the
// C ABI that bench.py / anx.parallel.workloads drive.
//
// One step over a hybrid batch x rows plan (anx/plan.hpp):
//   scatter   root X[images, tile.in rows] -> every rank's Tile             (root input only: io stream)
//   stage1    conv1 + ReLU + pool1 into the conv2 window, chunk by chunk   (compute stream)
//   halo_p1   pool1 rows between row neighbours, one transfer list per chunk (halo stream), so the
//             halo of chunk c moves while stage1 computes chunk c+1 and stage2(c) waits only for it
//   stage2    conv2 + ReLU + pool2 + LRN of each chunk                      (compute stream)
//   gather    Y[images, tile.out rows] -> root YFull                        (transport, io stream)
// With local input (the default, BASELINE.json's "device-resident RCCL/xGMI halo + gather") every
// rank's images x input rows live on its device from set_input on: a step moves only halos and the
// gather. A rank whose tile needs no halo (a row group of one rank, or overlap tiles) runs its images
// as free-running stream lanes (the fused tile forward on each), joined only by the gather. Steady
// state is pipelined across steps: scatter(k+1) and gather(k) run on the io stream while the compute
// streams run step k; no stream is synchronised with the host inside a step. Weights reach every rank
// by a device broadcast from the root (reference M4/M5 MPI_Bcast, v4_mpi_cuda/src/main_mpi_cuda.cpp:47-50).
// The default row split is the cost model's (anx/cost.hpp), which weighs scatter / halo / gather bytes
// against per-rank compute.
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "anx/comm.hpp"
#include "anx/cost.hpp"
#include "anx/engine.hpp"
#include "anx/plan.hpp"
#include "anx/schedule.hpp"

namespace anx {

struct V5Options {
  int batch = 1024;
  // row split inside each group of ranks: -1 = the cost model's pick (anx/cost.hpp pick_row_ways), 0 =
  // batch first, rows only below one image per rank (make_hybrid_plan's auto), r > 0 = groups of r
  // ranks (np = the reference's pure row split)
  int row_ways = -1;
  Decomp mode = Decomp::PerLayer;
  // local (default): the BASELINE's device-resident V5 ("halo + gather"): every rank holds its images x
  // input rows on its own device (placed once by set_input), so a step moves only pool1 halos and the
  // gather; root: the reference's data flow, the root scatters the batch every step
  InputSource input_source = InputSource::Local;
  std::string transport = "auto";  // auto | rccl | peer | loopback (RCCL transport over the loopback comm)
  int chunks = 0;                  // halo pipeline chunks per step (0 = auto)
  int pipeline = -1;               // scatter(k+1) / gather(k) on the io stream: -1 auto, 0 off, 1 on
  int lanes = 2;                   // stream lanes for a rank whose tile needs no halo (whole images, overlap tiles)
  // batch split (one rank per group): rank 0's images, the rest split evenly over the peers -- the dp
  // headline's root shedding (rank 0 also receives the gather, bench.py / cost.hpp dp_root_batch);
  // -1 = an even split. Invalid with a row split.
  int root_images = -1;
  bool poison = false;             // NaN-fill every consumed buffer after use (ordering tests)
  bool keep_log = false;           // keep the transport's log of issued transfers (tests)
  std::string peer_sync;           // peer transport ordering: "" (default) | flags | notes
  std::string cost;                // cost-model overrides for the row-split pick ("name=value;...")
  Impl impl = Impl::Mfma;
  Knobs knobs = default_knobs();
  // CPU ranks (no HIP call at all): the host engine (CpuBlocks) and the host transport (HostComm
  // point-to-point) execute the same layout, schedule and phase order, serially per step; transport,
  // lanes, pipeline and poison do not apply. What the CPU multi-rank tests and bench.py --device cpu run.
  bool host = false;
};

// Decomposition quality of a plan: output rows per rank (max / mean, 1.0 = balanced) and the conv1
// rows computed twice (anx/plan.hpp conv1_redundancy; 0 for a pure batch split).
struct PlanStats {
  int groups = 1, row_ways = 1;
  double rows_max = 0, rows_mean = 0, imbalance = 1, conv1_redundancy = 0, images_max = 0;
};
PlanStats plan_stats(const HybridPlan& p);

// V5 transport by node: auto = RCCL when every rank of this node has its own GPU or the job spans
// nodes, else peer (IPC, ranks share a GPU); loopback = the RCCL transport over the loopback device
// comm (ranks share a GPU; single node). Throws for a combination that cannot run.
std::string pick_v5_transport(const std::string& want, const RankInfo& ri, int ndev, bool dry);

// The plan, schedule and halo chunking of a V5 job: identical on every rank (a pure function of the
// job shape), which is what keeps every rank's sequence of transport calls the same.
struct RankBytes {  // bytes one rank sends / receives per step, by phase
  double scatter_recv = 0, scatter_sent = 0, halo_sent = 0, halo_recv = 0, gather_sent = 0, gather_recv = 0;
};
struct V5Layout {
  HybridPlan plan;
  Schedule sched;
  int row_ways = 1, chunks = 1;
  bool local_input = true;                          // no scatter inside a step (placed once by set_input)
  std::vector<std::vector<Transfer>> halo_chunks;  // chunk_of(P1Halo list, c, chunks)
  // every transfer of one step in issue order: scatter (root input only), halo chunks, gather
  std::vector<Transfer> step_transfers() const;
  // per rank, from step_transfers(); input_placement_bytes: the one-time placement of local input
  std::vector<RankBytes> rank_bytes() const;
  double input_placement_bytes() const;
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
  // following step (other ranks pass nullptr). Drains the pipeline first. Local input: the images x
  // rows of every rank are placed on its device here, once (not part of a step).
  void set_input(const float* host_x);
  // Enqueue one step (pipelined with its neighbours when the pipeline is on). No host sync.
  void step();
  // Wait for every enqueued step on every stream of this rank.
  void sync();
  // Fail-stop after an error on this rank (not collective): the transport releases every device-side
  // wait on a peer (ncclCommAbort / raised flag words), so the destructor's device sync returns; the
  // collective teardown is skipped. Call before rethrowing; the runtime is unusable afterwards.
  void abort();
  // Root: the output of the last step [batch, Hp2, Wp2, C2] into host memory (syncs first).
  void output(float* host_y);
  // Mean ms per step since the last reset, by phase, on the compute stream's critical path:
  // scatter (waiting for the input), stage1, halo_p1 (waiting for halo chunks), stage2, gather
  // (end of stage2 to end of the gather), compute (= stage1 + halo_p1 + stage2; a rank without halos
  // runs its tile as free-running stream lanes and reports its span as stage2). Syncs first.
  std::vector<std::pair<std::string, double>> phase_ms();
  void reset_phases();

  const V5Layout& layout() const { return lay_; }
  PlanStats stats() const { return plan_stats(lay_.plan); }
  const char* transport() const;
  bool pipelined() const { return pipeline_; }
  long steps() const;
  std::string describe_json() const;
  // transfers this rank's transport issued since construction (V5Options::keep_log)
  std::vector<std::string> transfer_log() const;

 private:
  struct Impl_;
  struct HostImpl_;
  std::unique_ptr<Impl_> p_;
  std::unique_ptr<HostImpl_> h_;  // V5Options::host
  V5Layout lay_;
  bool pipeline_ = false;
};

// Record-only schedule of rank `rank` of `np` (no GPU, no communication): the transfers its transport
// would issue in one step, in issue order (--dry-run, tests).
std::vector<std::string> v5_dry_schedule(int rank, int np, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
                                         const V5Options& o, const std::string& transport);

}  // namespace anx
