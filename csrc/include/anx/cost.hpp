// anx/cost.hpp — step-time cost model of the multi-GPU workloads (dp, V4, V5) and the comm-aware
// choice of the row split it drives.
//
// The reference has no model of its own scaling; it measures np = 1/2/4 on one GPU and derives
// speedup S = T1 / Tnp and efficiency E = S / np afterwards (log_analysis.py:212-222). Only one GPU
// is reachable from this build's test boxes, so the 2/4/8-GPU curve is MODELLED from measured
// single-GPU inputs and labelled as such ("measured": false) wherever it is printed.
//
// One step of a workload over np ranks is priced from the hybrid batch x rows plan (anx/plan.hpp):
//   compute   per rank: images x (stage1 share x conv1 rows + stage2 share x conv2 rows) of the tile,
//             in whole-image equivalents, at the measured single-GPU rate for that many images
//             (CostParams::rate, interpolated in log2(images)); row tiles of the per-layer split pay
//             split_penalty (pool1 not fused into the Conv2 input transform, window materialised);
//             the root's compute slows by ingest_slowdown (per 155 MB received per step) while it
//             receives the gather (measured on one GPU by tools/probe_ingest.py); in dp the root then
//             takes a proportionally smaller share of the images (dp_root_shed).
//   egress    root -> peers (the scatter of a root-held batch): each peer's bytes over its own xGMI
//             link, all links in parallel: max over peers / xgmi_gbps.
//   ingress   peers -> root (the output gather): likewise.
//   halo      per-layer pool1 halos: the busiest rank's halo bytes over one link; with C chunks only
//             1/C of it is exposed (halo c moves while stage1 computes chunk c+1) plus a per-phase
//             latency per chunk.
//   h2d/d2h   V4: every rank DMAs its own images x input rows from the shared host segment over its
//             own host link (h2d_gbps), bounded in aggregate by host memory (host_gbps); chunked and
//             pipelined across steps (H2D of step k+1 runs under step k's last chunks), so a step costs
//             the slowest stage plus v4_fill of the other two (0.1: 256 images at N=1 measured 2.94 ms
//             against an H2D stage of 2.79 ms, profiles/r03_v4_chunks.jsonl).
// Pipelined workloads (dp's gather overlapped with the next step; V5's io stream carrying scatter
// (k+1) then gather (k) beside step k's compute) cost max(compute + exposed halo, io); the bound is
// the term that sets the step.
#pragma once
#include <string>
#include <vector>

#include "anx/plan.hpp"

namespace anx {

enum class Workload : int { DP = 0, V4 = 1, V5 = 2 };
enum class InputSource : int { Local = 0, Root = 1 };

struct CostParams {
  // measured single-GPU throughput of the fp32 Blocks 1-2 engine (free-running stream lanes, one
  // lane below 32 images), images per GPU -> images/s, medians of tools/sweep_batch.py
  // (profiles/r06_final/sweep_lanes2_async.log, round 6 kernels; the bench step itself runs 350 k at 128)
  std::vector<int> rate_images{1, 8, 16, 32, 64, 128, 256, 512, 1024};
  std::vector<double> rate_img_s{11670, 55230, 140770, 197410, 286340, 330520, 332330, 335570, 327790};
  double min_step_ms = 0.08;     // a forward's kernel chain never takes less (batch 1: 0.081 ms, r01_algo_crossover)
  double stage1_share = 0.37;    // conv1 (+ its transform) share of one image's kernel time (r03 kernel table)
  double split_penalty = 1.03;   // per-layer row tiles: unfused pool1 + window (profiles/r03_fuse_pool1_bench_ab)
  double xgmi_gbps = 50.0;       // one xGMI link, one direction, as RCCL P2P sees it (assumed; not measurable here)
  double h2d_gbps = 56.7;        // one GPU's host link, measured (profiles/r03_v4_chunks.jsonl)
  double d2h_gbps = 56.7;        // assumed equal to H2D
  double host_gbps = 400.0;      // host memory feeding all H2D streams at once (assumed)
  // root compute slowdown while it receives the gather, per 155.06 MB per step (the dp N=8 volume),
  // linear in the bytes received: 0.15 measured by tools/probe_ingest.py (the bench step beside a
  // 155 MB/step receive-side copy: +11 % on all CUs, +18 % on 64 workgroups; profiles/r04_probe_ingest.jsonl)
  double ingest_slowdown = 0.15;
  int dp_root_shed = 1;          // dp: the root computes B / (1 + its slowdown) images (even), the peers B
  double phase_latency_ms = 0.02;  // per transport phase (RCCL group launch / flag round trip)
  double v4_fill = 0.1;          // exposed share of V4's non-bottleneck stages (see above)
  int v5_chunks = 0;             // V5 halo chunks (0 = the runtime's auto rule)
};

struct StepCost {
  Workload wl = Workload::DP;
  int np = 1, batch = 1, row_ways = 1, groups = 1;
  InputSource src = InputSource::Local;
  Decomp mode = Decomp::PerLayer;
  double compute_ms = 0, egress_ms = 0, ingress_ms = 0, halo_ms = 0, halo_exposed_ms = 0, h2d_ms = 0, d2h_ms = 0;
  double step_ms = 0, images_per_s = 0;
  // bytes per step
  double root_egress_bytes = 0, root_ingress_bytes = 0, max_peer_egress_bytes = 0, max_peer_ingress_bytes = 0;
  double max_rank_h2d_bytes = 0, max_rank_d2h_bytes = 0, total_h2d_bytes = 0, max_rank_halo_bytes = 0;
  double max_rank_work = 0;  // whole-image equivalents of the busiest rank
  int root_batch = 0;        // images the root computes per step (dp: after shedding)
  int images = 0;            // images per step over all ranks
  std::string bound;         // compute | egress | ingress | io | halo | h2d | d2h | host
  std::string json() const;
};

// dp: `batch` = images per GPU (weak scaling; a step moves np x batch images, less the root's shed
// share); v4 / v5: the global batch (strong scaling). row_ways: as make_hybrid_plan (0 = batch first) or -1 = pick_row_ways.
StepCost model_step(Workload wl, int np, int batch, int row_ways, InputSource src, Decomp mode,
                    const CostParams& p = CostParams{}, const BlockSpec& b1 = kBlock1, const BlockSpec& b2 = kBlock2,
                    int H = kInH, int W = kInW);

// CostParams from "name=value;..." overrides of the defaults (names: the fields above; rate=IMG:IPS,IMG:IPS,...
// replaces the rate table). Throws std::invalid_argument for an unknown name or a malformed value.
CostParams cost_params(const std::string& overrides);

// dp: images the root computes per step when every rank has `batch` (its ingest slowdown shed; even,
// so two lanes split it equally); = batch when shedding is off or np == 1.
int dp_root_batch(int np, int batch, const CostParams& p = CostParams{}, int H = kInH, int W = kInW);

// The row split with the lowest modelled step over the divisors r of np (ties: fewer row ways). For V4
// this is the batch split whenever the step is H2D-bound (a row split adds the rows' receptive-field
// overlap to every rank's H2D); for V5 it weighs scatter / halo / gather bytes against compute balance.
int pick_row_ways(Workload wl, int np, int batch, InputSource src, Decomp mode, const CostParams& p = CostParams{},
                  const BlockSpec& b1 = kBlock1, const BlockSpec& b2 = kBlock2, int H = kInH, int W = kInW);

// Modelled scaling curve over nps (e.g. 1, 2, 4, 8): per N the chosen row split, step, throughput,
// bound, speedup S = T(1) / T(N) (strong) or X(N) / X(1) (dp), efficiency S / N. JSON object with
// "measured": false.
std::string model_curve_json(Workload wl, const std::vector<int>& nps, int batch, int row_ways, InputSource src,
                             Decomp mode, const CostParams& p = CostParams{});

}  // namespace anx
