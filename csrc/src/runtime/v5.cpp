// V5 runtime: device-resident scatter -> stage1 -> chunked pool1 halos -> stage2 -> gather (anx/v5.hpp).
#include "anx/v5.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "anx/cpu_engine.hpp"
#include "anx/trace.hpp"

namespace anx {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("v5 ") + what + ": " + hipGetErrorString(e));
}
constexpr int kB = static_cast<int>(BufId::kCount);
constexpr int kMaxChunks = 16;  // the peer transport's halo channels
constexpr int kRing = 32;       // per-step timing event sets kept before they are folded in
constexpr int kMaxLanes = 4;
constexpr int kLaneMin = 16;    // images per lane below which a rank keeps one lane (Winograd needs > 8)
const char* kPhase[5] = {"scatter", "stage1", "halo_p1", "stage2", "gather"};
}  // namespace

PlanStats plan_stats(const HybridPlan& p) {
  PlanStats s;
  s.groups = p.groups;
  double work_sum = 0, work_max = 0, rows_sum = 0;
  for (int r = 0; r < p.np; ++r) {
    const TilePlan& t = p.tile(r);
    const int rows = t.out.size();
    const int imgs = rows ? p.images[p.group_of[r]].size() : 0;
    s.row_ways = std::max(s.row_ways, p.group_size[p.group_of[r]]);
    rows_sum += rows;
    s.rows_max = std::max(s.rows_max, static_cast<double>(rows));
    s.images_max = std::max(s.images_max, static_cast<double>(imgs));
    work_sum += static_cast<double>(rows) * imgs;
    work_max = std::max(work_max, static_cast<double>(rows) * imgs);
  }
  s.rows_mean = rows_sum / p.np;
  s.imbalance = work_sum > 0 ? work_max / (work_sum / p.np) : 1.0;
  s.conv1_redundancy = conv1_redundancy(p);
  return s;
}

std::string pick_v5_transport(const std::string& want, const RankInfo& ri, int ndev, bool dry) {
  const bool shared = !dry && ri.local_world > ndev;  // ranks of this node outnumber its GPUs
  const std::string tr = want == "auto" ? (shared && ri.nnodes == 1 ? "peer" : "rccl") : want;
  if (tr != "rccl" && tr != "peer" && tr != "loopback")
    throw std::runtime_error("--transport must be auto, rccl, peer or loopback");
  if ((tr == "peer" || tr == "loopback") && ri.nnodes > 1)
    throw std::runtime_error("the " + tr + " transport (IPC) is single-node: use --transport rccl across nodes");
  if (tr == "rccl" && shared)
    throw std::runtime_error("v5 over RCCL needs one GPU per rank on each node (" + std::to_string(ri.local_world) +
                             " ranks, " + std::to_string(ndev) + " GPUs here; --transport peer shares a GPU)");
  return tr;
}

V5Layout make_v5_layout(int np, const BlockSpec& b1, const BlockSpec& b2, int H, int W, const V5Options& o) {
  V5Layout L;
  L.local_input = o.input_source == InputSource::Local;
  L.row_ways = o.row_ways < 0
                   ? pick_row_ways(Workload::V5, np, o.batch, o.input_source, o.mode, cost_params(o.cost), b1, b2, H, W)
                   : o.row_ways;
  if (!make_hybrid_plan(H, W, np, o.batch, L.row_ways, o.mode, L.plan, b1, b2))
    throw std::runtime_error("v5: invalid plan (row_ways " + std::to_string(L.row_ways) + " over " +
                             std::to_string(np) + " ranks)");
  if (o.root_images >= 0 && np > 1) {  // root shedding: rank 0 takes root_images, the peers the rest evenly
    HybridPlan& p = L.plan;
    if (p.groups != np || o.root_images < 1 || o.batch - o.root_images < np - 1)
      throw std::runtime_error("v5: root_images " + std::to_string(o.root_images) + " needs a batch split with >= 1 image "
                               "per rank (" + std::to_string(o.batch) + " images over " + std::to_string(np) + " ranks)");
    p.images[0] = RowRange{0, o.root_images};
    const std::vector<RowRange> rest = split_rows(o.batch - o.root_images, np - 1);
    for (int g = 1; g < np; ++g) p.images[g] = RowRange{o.root_images + rest[g - 1].lo, o.root_images + rest[g - 1].hi};
  }
  const BlocksDims d = blocks_dims(H, W, b1, b2);
  const size_t in_row = static_cast<size_t>(d.W) * d.C0 * 4, out_row = static_cast<size_t>(d.Wp2) * d.C2 * 4;
  const size_t win_row = static_cast<size_t>(d.Wp1 + 2 * b2.conv.P) * d.C1 * 4;
  L.sched = make_step_schedule(L.plan, {in_row, out_row, win_row, d.H, d.Hp2});
  const auto& halos = L.sched.phase[static_cast<int>(Phase::P1Halo)];
  int min_imgs = 1 << 30;
  for (const Transfer& x : halos) min_imgs = std::min(min_imgs, static_cast<int>(x.height));
  // auto: one chunk. Chunking (halo c moves while stage1 computes c+1) never paid: at the BASELINE
  // share (256 images per 2-way row group) 1.207 vs 1.226 ms at np 2 and 2.645 vs 2.646 ms at np 4 for
  // 1 vs 2 chunks, stage1's smaller launches losing what the hidden halo gains
  // (profiles/r04_halo/, profiles/r03_v5_halo.log); --chunks K keeps the pipeline for other links
  const int auto_chunks = 1;
  L.chunks = halos.empty() ? 1 : std::max(1, std::min({o.chunks > 0 ? o.chunks : auto_chunks, min_imgs, kMaxChunks}));
  for (int c = 0; c < L.chunks; ++c) L.halo_chunks.push_back(chunk_of(halos, c, L.chunks));
  return L;
}

std::vector<Transfer> V5Layout::step_transfers() const {
  std::vector<Transfer> v;
  if (!local_input) v = sched.phase[static_cast<int>(Phase::Scatter)];
  for (const auto& c : halo_chunks) v.insert(v.end(), c.begin(), c.end());
  const auto& g = sched.phase[static_cast<int>(Phase::Gather)];
  v.insert(v.end(), g.begin(), g.end());
  return v;
}

std::vector<RankBytes> V5Layout::rank_bytes() const {
  std::vector<RankBytes> b(plan.np);
  for (const Transfer& x : step_transfers()) {
    if (x.src == x.dst) continue;
    const double n = static_cast<double>(x.bytes());
    switch (x.phase) {
      case Phase::Scatter: b[x.src].scatter_sent += n, b[x.dst].scatter_recv += n; break;
      case Phase::P1Halo: b[x.src].halo_sent += n, b[x.dst].halo_recv += n; break;
      case Phase::Gather: b[x.src].gather_sent += n, b[x.dst].gather_recv += n; break;
    }
  }
  return b;
}

double V5Layout::input_placement_bytes() const {
  double n = 0;
  if (local_input)
    for (const Transfer& x : sched.phase[static_cast<int>(Phase::Scatter)])
      if (x.src != x.dst) n += static_cast<double>(x.bytes());
  return n;
}

std::vector<std::string> v5_dry_schedule(int rank, int np, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
                                         const V5Options& o, const std::string& transport) {
  const V5Layout L = make_v5_layout(np, b1, b2, H, W, o);
  std::unique_ptr<Transport> x = transport == "peer" ? make_peer_transport(nullptr, 0, rank, o.peer_sync)
                                                     : make_rccl_transport(nullptr, 0, rank, transport == "loopback");
  x->record_only = true;
  void* none[2][kB] = {};
  x->bind(L.sched, none, nullptr);
  if (!L.local_input) x->run_phase(Phase::Scatter, L.sched.phase[0], nullptr, 0);
  for (const auto& c : L.halo_chunks) x->run_phase(Phase::P1Halo, c, nullptr, 0);
  x->run_phase(Phase::Gather, L.sched.phase[2], nullptr, 0);
  return x->log();
}

// ------------------------------------------------------------------------------------------ runtime
struct V5Runtime::Impl_ {
  HostComm& c;
  RankInfo ri;
  V5Options o;
  const V5Layout& L;
  BlocksDims d;
  int rank = 0, np = 1, dev = 0, C = 1;
  std::string tr;
  std::unique_ptr<Transport> x;
  std::unique_ptr<BlocksEngine> eng;
  TilePlan t;
  int n = 0;  // images this rank computes
  // lane path: a tile that needs no halo (a row group of one rank, or overlap tiles) runs as nl
  // free-running stream lanes, lane i images [lb[i], lb[i+1]) on engine leng[i] / stream ls[i]
  // (lane 0 = eng on st); only the gather joins them
  bool lane_path = false, local = true;
  int nl = 1;  // lanes
  std::vector<int> lb;
  std::vector<std::unique_ptr<BlocksEngine>> leng;
  std::vector<hipStream_t> ls;
  hipEvent_t e_lane[kMaxLanes][2] = {}, e_go[2] = {}, e_gdone[2] = {};
  std::vector<int> lo;  // this rank's chunk bounds (C + 1)
  size_t x_bytes = 0, yfull_bytes = 0, tile_bytes = 0, y_bytes = 0;
  float* d_x = nullptr;
  float* d_tile[2] = {nullptr, nullptr};
  float* d_y[2] = {nullptr, nullptr};
  float* d_yfull[2] = {nullptr, nullptr};
  bool alias_tile = false, alias_y = false;
  std::vector<float*> owned;  // device allocations to free
  hipStream_t st = nullptr, io = nullptr, hs = nullptr;
  bool aborted = false;
  hipEvent_t e_sc[2] = {}, e_s2[2] = {}, e_hdone = nullptr;
  std::vector<hipEvent_t> e_s1, e_h;
  long k = 0;
  bool prefetched = false;
  bool pipeline = false;
  // timing: ring of per-step event sets (5 + 2 C events), folded into sums when reused or read
  std::vector<std::vector<hipEvent_t>> ring;
  std::vector<bool> pending;
  int ring_pos = 0;
  double sums[5] = {0, 0, 0, 0, 0};
  long timed = 0;

  Impl_(HostComm& cc, const RankInfo& r, const V5Options& oo, const V5Layout& l) : c(cc), ri(r), o(oo), L(l) {}

  float* dalloc(size_t bytes) {
    void* p = nullptr;
    hip_ok(hipMalloc(&p, std::max<size_t>(bytes, 4)), "hipMalloc");
    owned.push_back(static_cast<float*>(p));
    return static_cast<float*>(p);
  }
  hipEvent_t event(bool timing = false) {
    hipEvent_t e = nullptr;
    hip_ok(hipEventCreateWithFlags(&e, timing ? hipEventDefault : hipEventDisableTiming), "hipEventCreate");
    return e;
  }
  void rec(hipEvent_t e, hipStream_t s) { hip_ok(hipEventRecord(e, s), "hipEventRecord"); }
  void wait(hipStream_t s, hipEvent_t e) { hip_ok(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent"); }

  void fold(int i) {  // accumulate the finished event set i
    if (!pending[i]) return;
    auto& e = ring[i];
    hip_ok(hipEventSynchronize(e.back()), "hipEventSynchronize");
    auto ms = [&](int a, int b) {
      float v = 0;
      hip_ok(hipEventElapsedTime(&v, e[a], e[b]), "hipEventElapsedTime");
      return static_cast<double>(v);
    };
    double halo = 0;
    for (int cc = 0; cc < C; ++cc) halo += ms(3 + 2 * cc, 4 + 2 * cc);
    sums[0] += ms(0, 1);
    sums[1] += ms(1, 2);
    sums[2] += halo;
    sums[3] += ms(2, 3 + 2 * C) - halo;
    sums[4] += ms(3 + 2 * C, 4 + 2 * C);
    ++timed;
    pending[i] = false;
  }

  void scatter(long kk, hipStream_t on) {
    RoctxRange r("v5 scatter");
    x->run_phase(Phase::Scatter, L.sched.phase[0], on, static_cast<int>(kk & 1));
  }
  void gather(long kk, hipStream_t on) {
    const int par = static_cast<int>(kk & 1);
    {
      RoctxRange r("v5 gather");
      x->run_phase(Phase::Gather, L.sched.phase[2], on, par);
    }
    if (o.poison && n && !alias_y) hip_ok(hipMemsetAsync(d_y[par], 0xff, y_bytes, on), "poison y");
  }
  BlocksEngine& lane_engine(int i) { return i == 0 ? *eng : *leng[i - 1]; }
  // Lane path: every lane waits for its step's input (`in_ev`: the scatter / the previous gather of
  // this parity, both on io; or e_go on st when not pipelined) on its own stream and runs the fused
  // tile forward of its slice; e_lane[i][par] marks it done (the gather waits for all of them).
  void compute_lanes(long kk, std::vector<hipEvent_t>& e, hipEvent_t in_ev) {
    const int par = static_cast<int>(kk & 1);
    rec(e[2], st);
    for (int cc = 0; cc < C; ++cc) rec(e[3 + 2 * cc], st), rec(e[4 + 2 * cc], st);  // no halo on this path
    const size_t in_img = n ? tile_bytes / n : 0, out_img = n ? y_bytes / n : 0;
    for (int i = 0; i < nl; ++i) {
      hipStream_t s = ls[i];
      const int a = lb[i], b = lb[i + 1];
      if (i > 0 && in_ev) wait(s, in_ev);
      if (b > a) {
        RoctxRange r("v5 lane tile");
        hip_ok(lane_engine(i).tile_forward(reinterpret_cast<float*>(reinterpret_cast<char*>(d_tile[par]) + a * in_img),
                                           b - a, t,
                                           reinterpret_cast<float*>(reinterpret_cast<char*>(d_y[par]) + a * out_img), s),
               "tile_forward");
        if (o.poison && !local && !alias_tile)
          hip_ok(hipMemsetAsync(reinterpret_cast<char*>(d_tile[par]) + a * in_img, 0xff, (b - a) * in_img, s),
                 "poison tile");
      }
      rec(e_lane[i][par], s);
    }
  }
  // make `s` wait for every lane of step parity `par`
  void join_lanes(hipStream_t s, int par) {
    for (int i = 0; i < nl; ++i) wait(s, e_lane[i][par]);
  }

  // stage1 chunks, halo chunks on hs, stage2 chunks; e: this step's timing events
  void compute(long kk, std::vector<hipEvent_t>& e) {
    const int par = static_cast<int>(kk & 1);
    const bool per_layer = o.mode == Decomp::PerLayer;
    // the previous step's halo pushes read this rank's window: stage1 may rewrite it only after them
    wait(st, e_hdone);
    for (int cc = 0; cc < C && per_layer; ++cc) {
      if (n && lo[cc + 1] > lo[cc]) {
        RoctxRange r("v5 stage1");
        hip_ok(eng->stage1(d_tile[par], n, t, st, lo[cc], lo[cc + 1]), "stage1");
        if (o.poison && !alias_tile && !local) {
          const size_t img = tile_bytes / n;
          hip_ok(hipMemsetAsync(reinterpret_cast<char*>(d_tile[par]) + lo[cc] * img, 0xff, (lo[cc + 1] - lo[cc]) * img,
                                st),
                 "poison tile");
        }
      }
      rec(e_s1[cc], st);
      wait(hs, e_s1[cc]);
      {
        RoctxRange r("v5 halo_p1");
        x->run_phase(Phase::P1Halo, L.halo_chunks[cc], hs, par);
      }
      rec(e_h[cc], hs);
    }
    rec(e_hdone, hs);
    rec(e[2], st);
    for (int cc = 0; cc < C; ++cc) {
      rec(e[3 + 2 * cc], st);
      if (per_layer) wait(st, e_h[cc]);
      rec(e[4 + 2 * cc], st);
      if (!n || lo[cc + 1] <= lo[cc]) continue;
      RoctxRange r("v5 stage2");
      {
        hip_ok(eng->stage2(n, t, d_y[par], st, lo[cc], lo[cc + 1]), "stage2");
        if (o.poison)  // the halo rows this rank received: the next step must bring them again
          for (const Transfer& h : L.halo_chunks[cc])
            if (h.dst == rank && h.src != rank)
              hip_ok(hipMemset2DAsync(reinterpret_cast<char*>(eng->q2_row_ptr(t, 0, t.q.lo)) + h.to.off, h.to.pitch,
                                      0xff, h.width, h.height, st),
                     "poison window");
      }
    }
    rec(e[3 + 2 * C], st);
  }
};

// ------------------------------------------------------------------------------------------ host
// V5Options::host: CPU ranks run the same layout (plan, schedule, halo chunks) through the host
// transport, one phase after another: scatter (root input), stage1, every halo chunk, stage2 (or the
// whole-tile forward where no halo touches the rank), gather. Phase times are host wall clock.
struct V5Runtime::HostImpl_ {
  HostComm& c;
  V5Options o;
  const V5Layout& L;
  BlocksDims d;
  int rank = 0, np = 1;
  std::unique_ptr<Transport> x;
  std::unique_ptr<CpuBlocks> eng;
  TilePlan t;
  int n = 0;
  bool lane_path = false, local = true;
  std::vector<float> X, tile[2], y[2], yfull[2];
  long k = 0, timed = 0;
  double sums[5] = {0, 0, 0, 0, 0};
  HostImpl_(HostComm& cc, const V5Options& oo, const V5Layout& l) : c(cc), o(oo), L(l) {}

  void init(const BlockSpec& b1, const BlockSpec& b2, int H, int W, const HostWeights& w) {
    rank = c.rank();
    np = c.size();
    d = blocks_dims(H, W, b1, b2);
    x = make_host_transport(&c, rank);
    x->keep_log = o.keep_log;
    local = L.local_input;
    HostWeights hw;  // the root's weights, broadcast over the transport (the reference's MPI_Bcast, M4/M5)
    init_const(hw, b1, b2);
    if (rank == 0) {
      if (w.w1.size() != hw.w1.size() || w.b1.size() != hw.b1.size() || w.w2.size() != hw.w2.size() ||
          w.b2.size() != hw.b2.size())
        throw std::runtime_error("v5: weight sizes do not match the block specs");
      hw = w;
    }
    for (std::vector<float>* v : {&hw.w1, &hw.b1, &hw.w2, &hw.b2}) x->bcast(v->data(), v->size() * 4, 0);
    const HybridPlan& hp = L.plan;
    t = hp.tile(rank);
    const RowRange im = hp.images[hp.group_of[rank]];
    n = t.out.empty() ? 0 : im.size();
    lane_path = o.mode == Decomp::Overlap || hp.group_size[hp.group_of[rank]] == 1;
    eng = std::make_unique<CpuBlocks>(b1, b2, H, W, hw);
    const size_t in_img = static_cast<size_t>(H) * W * d.C0, out_img = static_cast<size_t>(d.Hp2) * d.Wp2 * d.C2;
    if (rank == 0) {
      X.assign(static_cast<size_t>(o.batch) * in_img, 0.f);
      for (auto& v : yfull) v.assign(static_cast<size_t>(o.batch) * out_img, 0.f);
    }
    for (int p = 0; p < 2; ++p) {
      tile[p].assign(std::max<size_t>(1, static_cast<size_t>(n) * t.in.size() * W * d.C0), 0.f);
      y[p].assign(std::max<size_t>(1, static_cast<size_t>(n) * t.out.size() * d.Wp2 * d.C2), 0.f);
    }
    float* win = nullptr;  // the conv2 window exists (and keeps its address) once stage1 has run
    if (n && !lane_path) {
      eng->stage1(tile[0].data(), n, t);
      win = eng->window_row(t, 0, t.q.lo);
    }
    void* bufs[2][kB];
    for (int p = 0; p < 2; ++p) {
      bufs[p][static_cast<int>(BufId::X)] = X.empty() ? nullptr : X.data();
      bufs[p][static_cast<int>(BufId::Tile)] = tile[p].data();
      bufs[p][static_cast<int>(BufId::Win)] = win;
      bufs[p][static_cast<int>(BufId::Y)] = y[p].data();
      bufs[p][static_cast<int>(BufId::YFull)] = yfull[p].empty() ? nullptr : yfull[p].data();
    }
    x->bind(L.sched, bufs, nullptr);
    c.barrier();
  }
  static double now() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void step() {
    const int par = static_cast<int>(k & 1);
    double t0 = now();
    if (!local) x->run_phase(Phase::Scatter, L.sched.phase[0], nullptr, par);
    const double t1 = now();
    if (n && !lane_path) eng->stage1(tile[par].data(), n, t);
    const double t2 = now();
    if (!lane_path)
      for (const auto& ch : L.halo_chunks) x->run_phase(Phase::P1Halo, ch, nullptr, par);
    const double t3 = now();
    if (n) {
      if (lane_path)
        eng->tile_forward(tile[par].data(), n, t, y[par].data());
      else
        eng->stage2(n, t, y[par].data());
    }
    const double t4 = now();
    x->run_phase(Phase::Gather, L.sched.phase[2], nullptr, par);
    const double t5 = now();
    const double v[5] = {t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4};
    for (int i = 0; i < 5; ++i) sums[i] += v[i];
    ++timed;
    ++k;
  }
};

V5Runtime::V5Runtime(HostComm& c, const RankInfo& ri, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
                     const HostWeights& w, const V5Options& o)
    : lay_(make_v5_layout(c.size(), b1, b2, H, W, o)) {
  if (o.host) {  // CPU ranks: no HIP call anywhere on this path
    h_ = std::make_unique<HostImpl_>(c, o, lay_);
    h_->init(b1, b2, H, W, w);
    pipeline_ = false;
    return;
  }
  p_ = std::make_unique<Impl_>(c, ri, o, lay_);
  Impl_& I = *p_;
  I.rank = c.rank();
  I.np = c.size();
  I.C = lay_.chunks;
  I.d = blocks_dims(H, W, b1, b2);
  int ndev = 0;
  hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  if (ndev < 1) throw std::runtime_error("v5 needs a GPU");
  I.tr = pick_v5_transport(o.transport, ri, ndev, false);
  I.dev = ri.local_rank % ndev;
  hip_ok(hipSetDevice(I.dev), "hipSetDevice");
  I.x = I.tr == "peer" ? make_peer_transport(&c, I.dev, I.rank, o.peer_sync)
                       : make_rccl_transport(&c, I.dev, I.rank, I.tr == "loopback");
  I.x->keep_log = o.keep_log;
  pipeline_ = I.pipeline = o.pipeline < 0 ? I.tr != "peer" : o.pipeline > 0;
  I.local = lay_.local_input;

  // weights: the root's host copy -> its device -> every rank's device (transport broadcast) -> host
  // (the engine packs / Winograd-transforms them once on the host)
  HostWeights hw;
  init_const(hw, b1, b2);
  const size_t nw[4] = {hw.w1.size(), hw.b1.size(), hw.w2.size(), hw.b2.size()};
  const size_t total = nw[0] + nw[1] + nw[2] + nw[3];
  if (I.rank == 0) {
    if (w.w1.size() != nw[0] || w.b1.size() != nw[1] || w.w2.size() != nw[2] || w.b2.size() != nw[3])
      throw std::runtime_error("v5: weight sizes do not match the block specs");
    hw = w;
  }
  if (I.np > 1) {
    void* wd = nullptr;
    hip_ok(hipMalloc(&wd, total * 4), "hipMalloc weights");
    std::vector<float>* parts[4] = {&hw.w1, &hw.b1, &hw.w2, &hw.b2};
    size_t off = 0;
    if (I.rank == 0)
      for (auto* v : parts) {
        hip_ok(hipMemcpy(static_cast<float*>(wd) + off, v->data(), v->size() * 4, hipMemcpyHostToDevice), "H2D weights");
        off += v->size();
      }
    I.x->bcast(wd, total * 4, 0);
    off = 0;
    if (I.rank != 0)
      for (auto* v : parts) {
        hip_ok(hipMemcpy(v->data(), static_cast<float*>(wd) + off, v->size() * 4, hipMemcpyDeviceToHost), "D2H weights");
        off += v->size();
      }
    hip_ok(hipFree(wd), "hipFree");
  }

  const HybridPlan& hp = lay_.plan;
  I.t = hp.tile(I.rank);
  const RowRange im = hp.images[hp.group_of[I.rank]];
  I.n = I.t.out.empty() ? 0 : im.size();
  for (int cc = 0; cc <= I.C; ++cc) I.lo.push_back(I.n * cc / I.C);
  // no halo touches this rank: its tile runs as free-running stream lanes of the fused forward
  I.lane_path = o.mode == Decomp::Overlap || hp.group_size[hp.group_of[I.rank]] == 1;
  I.nl = I.lane_path ? std::max(1, std::min({o.lanes, kMaxLanes, I.n / kLaneMin})) : 1;
  for (int i = 0; i <= I.nl; ++i) I.lb.push_back(I.n * i / I.nl);
  I.eng = std::make_unique<BlocksEngine>(b1, b2, H, W, hw, std::max(1, I.lb[1] - I.lb[0]), o.impl, o.knobs);
  for (int i = 1; i < I.nl; ++i)
    I.leng.push_back(std::make_unique<BlocksEngine>(b1, b2, H, W, hw, std::max(1, I.lb[i + 1] - I.lb[i]), o.impl, o.knobs));
  hip_ok(hipStreamCreateWithFlags(&I.st, hipStreamNonBlocking), "hipStreamCreate");
  hip_ok(hipStreamCreateWithFlags(&I.io, hipStreamNonBlocking), "hipStreamCreate");
  hip_ok(hipStreamCreateWithFlags(&I.hs, hipStreamNonBlocking), "hipStreamCreate");
  I.ls.push_back(I.st);
  for (int i = 1; i < I.nl; ++i) {
    hipStream_t s = nullptr;
    hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    I.ls.push_back(s);
  }

  const BlocksDims& d = I.d;
  const size_t in_img = static_cast<size_t>(H) * W * d.C0 * 4, out_img = static_cast<size_t>(d.Hp2) * d.Wp2 * d.C2 * 4;
  I.tile_bytes = static_cast<size_t>(I.n) * I.t.in.size() * W * d.C0 * 4;
  I.y_bytes = static_cast<size_t>(I.n) * I.t.out.size() * d.Wp2 * d.C2 * 4;
  if (I.rank == 0) {
    I.x_bytes = static_cast<size_t>(o.batch) * in_img;
    I.yfull_bytes = static_cast<size_t>(o.batch) * out_img;
    I.d_x = I.dalloc(I.x_bytes);
    hip_ok(hipMemset(I.d_x, 0, I.x_bytes), "hipMemset");
    for (auto& y : I.d_yfull) y = I.dalloc(I.yfull_bytes);
  }
  // the root's whole-image tiles are computed in place inside X / YFull (no local copies)
  I.alias_tile = I.rank == 0 && I.n && I.t.in.size() == H;
  I.alias_y = I.rank == 0 && I.n && I.t.out.size() == d.Hp2;
  for (int p = 0; p < 2; ++p) {
    I.d_tile[p] = I.alias_tile ? reinterpret_cast<float*>(reinterpret_cast<char*>(I.d_x) + im.lo * in_img)
                               : I.dalloc(I.tile_bytes);
    I.d_y[p] = I.alias_y ? reinterpret_cast<float*>(reinterpret_cast<char*>(I.d_yfull[p]) + im.lo * out_img)
                         : I.dalloc(I.y_bytes);
  }
  // the conv2 window exists once stage1 has seen this tile geometry: run it once on zeros
  float* d_win = nullptr;
  if (I.n && !I.lane_path) {
    if (!I.alias_tile) hip_ok(hipMemsetAsync(I.d_tile[0], 0, I.tile_bytes, I.st), "hipMemset");
    hip_ok(I.eng->stage1(I.d_tile[0], I.n, I.t, I.st), "stage1");
    d_win = I.eng->q2_row_ptr(I.t, 0, I.t.q.lo);
  }
  hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  void* bufs[2][kB];
  for (int p = 0; p < 2; ++p) {
    bufs[p][static_cast<int>(BufId::X)] = I.d_x;
    bufs[p][static_cast<int>(BufId::Tile)] = I.d_tile[p];
    bufs[p][static_cast<int>(BufId::Win)] = d_win;
    bufs[p][static_cast<int>(BufId::Y)] = I.d_y[p];
    bufs[p][static_cast<int>(BufId::YFull)] = I.d_yfull[p];
  }
  I.x->bind(lay_.sched, bufs, I.st);
  for (int p = 0; p < 2; ++p) {
    I.e_sc[p] = I.event(), I.e_s2[p] = I.event(), I.e_go[p] = I.event(), I.e_gdone[p] = I.event();
    for (int i = 0; i < I.nl; ++i) I.e_lane[i][p] = I.event();
  }
  I.e_hdone = I.event();
  for (int cc = 0; cc < I.C; ++cc) I.e_s1.push_back(I.event()), I.e_h.push_back(I.event());
  I.ring.resize(kRing);
  for (auto& e : I.ring)
    for (int i = 0; i < 5 + 2 * I.C; ++i) e.push_back(I.event(true));
  I.pending.assign(kRing, false);
  c.barrier();
}

V5Runtime::~V5Runtime() {
  if (!p_) return;
  Impl_& I = *p_;
  (void)hipDeviceSynchronize();  // after abort() no stream waits on a peer any more
  try {
    if (!I.aborted) {
      I.c.barrier();  // nobody pushes into a peer's buffers any more
      I.x->close();   // collective: unmap, barrier, free own
    }
  } catch (...) {
  }
  I.x.reset();
  I.eng.reset();
  I.leng.clear();
  for (float* p : I.owned) (void)hipFree(p);
  for (int p = 0; p < 2; ++p) {
    for (hipEvent_t v : {I.e_go[p], I.e_gdone[p]})
      if (v) (void)hipEventDestroy(v);
    for (int i = 0; i < kMaxLanes; ++i)
      if (I.e_lane[i][p]) (void)hipEventDestroy(I.e_lane[i][p]);
  }
  for (size_t i = 1; i < I.ls.size(); ++i) (void)hipStreamDestroy(I.ls[i]);
  for (auto& e : I.ring)
    for (hipEvent_t v : e) (void)hipEventDestroy(v);
  for (hipEvent_t v : I.e_s1) (void)hipEventDestroy(v);
  for (hipEvent_t v : I.e_h) (void)hipEventDestroy(v);
  for (hipEvent_t v : {I.e_sc[0], I.e_sc[1], I.e_s2[0], I.e_s2[1], I.e_hdone})
    if (v) (void)hipEventDestroy(v);
  for (hipStream_t s : {I.st, I.io, I.hs})
    if (s) (void)hipStreamDestroy(s);
}

const char* V5Runtime::transport() const { return h_ ? h_->x->name() : p_->x->name(); }
long V5Runtime::steps() const { return h_ ? h_->k : p_->k; }

void V5Runtime::set_input(const float* host_x) {
  if (h_) {
    HostImpl_& I = *h_;
    if (I.rank == 0) {
      if (!host_x) throw std::runtime_error("v5 set_input: the root needs the batch");
      std::memcpy(I.X.data(), host_x, I.X.size() * 4);
    }
    if (I.local) {  // every rank's images x input rows placed once, in both step parities
      I.c.barrier();
      for (int par = 0; par < 2; ++par) I.x->run_phase(Phase::Scatter, lay_.sched.phase[0], nullptr, par);
    }
    I.c.barrier();
    return;
  }
  Impl_& I = *p_;
  sync();
  if (I.rank == 0) {
    if (!host_x) throw std::runtime_error("v5 set_input: the root needs the batch");
    hip_ok(hipMemcpy(I.d_x, host_x, I.x_bytes, hipMemcpyHostToDevice), "H2D input");
  }
  I.prefetched = false;  // every rank drops its prefetched scatter: the next step scatters again
  if (I.local) {
    // device-resident input: every rank's images x input rows land on its device now, in both step
    // parities' tile buffers; steps then move only halos and the gather
    I.c.barrier();  // the root's X is complete before anyone pulls from it
    for (int par = 0; par < 2; ++par) {
      RoctxRange r("v5 input placement");
      I.x->run_phase(Phase::Scatter, lay_.sched.phase[0], I.st, par);
    }
    hip_ok(hipStreamSynchronize(I.st), "hipStreamSynchronize");
  }
  I.c.barrier();
}

void V5Runtime::step() {
  if (h_) return h_->step();
  Impl_& I = *p_;
  const long k = I.k;
  const int par = static_cast<int>(k & 1);
  const int slot = I.ring_pos;
  I.fold(slot);
  std::vector<hipEvent_t>& e = I.ring[slot];
  I.ring_pos = (I.ring_pos + 1) % kRing;
  if (!I.pipeline) {  // every phase in step order on the compute stream (side lanes fork from it)
    I.rec(e[0], I.st);
    if (!I.local) I.scatter(k, I.st);
    I.rec(e[1], I.st);
    if (I.lane_path) {
      I.rec(I.e_go[par], I.st);
      I.compute_lanes(k, e, I.e_go[par]);
      I.join_lanes(I.st, par);
      I.rec(e[3 + 2 * I.C], I.st);
    } else {
      I.compute(k, e);
    }
    I.gather(k, I.st);
    I.rec(e.back(), I.st);
  } else {
    // io runs scatter(k+1) while the compute stream(s) run step k, then gather(k) once step k's
    // outputs are complete; compute starts step k+1 as soon as its input is there (scatter(k+1), or
    // with local input the gather that last read this parity's outputs). Every rank issues the phases
    // in the same order (scatter k+1, gather k), as RCCL's in-order matching and the peer flag
    // counters require.
    if (!I.local && !I.prefetched) {
      I.scatter(k, I.io);
      I.rec(I.e_sc[par], I.io);
    }
    hipEvent_t in_ev = I.local ? I.e_gdone[par] : I.e_sc[par];
    I.rec(e[0], I.st);
    I.wait(I.st, in_ev);
    I.rec(e[1], I.st);
    if (I.lane_path) {
      I.compute_lanes(k, e, in_ev);
    } else {
      I.compute(k, e);
      I.rec(I.e_s2[par], I.st);
    }
    if (!I.local) {
      I.scatter(k + 1, I.io);
      I.rec(I.e_sc[par ^ 1], I.io);
      I.prefetched = true;
    }
    if (I.lane_path) {
      I.join_lanes(I.io, par);
      I.rec(e[3 + 2 * I.C], I.io);
    } else {
      I.wait(I.io, I.e_s2[par]);
    }
    I.gather(k, I.io);
    I.rec(I.e_gdone[par], I.io);
    I.rec(e.back(), I.io);
  }
  I.pending[slot] = true;
  ++I.k;
}

void V5Runtime::abort() {
  if (!p_ || p_->aborted) return;  // host mode: every phase is complete on return, nothing is parked
  p_->aborted = true;
  if (p_->x) p_->x->abort();
}

void V5Runtime::sync() {
  if (h_) return;  // host mode: blocking phases
  Impl_& I = *p_;
  for (hipStream_t s : {I.st, I.io, I.hs}) hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
  for (size_t i = 1; i < I.ls.size(); ++i) hip_ok(hipStreamSynchronize(I.ls[i]), "hipStreamSynchronize");
}

std::vector<std::string> V5Runtime::transfer_log() const { return h_ ? h_->x->log() : p_->x->log(); }

void V5Runtime::output(float* host_y) {
  if (h_) {
    if (h_->rank != 0) return;
    if (h_->k == 0) throw std::runtime_error("v5 output: no step has run");
    const std::vector<float>& v = h_->yfull[(h_->k - 1) & 1];
    std::memcpy(host_y, v.data(), v.size() * 4);
    return;
  }
  Impl_& I = *p_;
  sync();
  if (I.rank != 0) return;
  if (I.k == 0) throw std::runtime_error("v5 output: no step has run");
  hip_ok(hipMemcpy(host_y, I.d_yfull[(I.k - 1) & 1], I.yfull_bytes, hipMemcpyDeviceToHost), "D2H output");
}

std::vector<std::pair<std::string, double>> V5Runtime::phase_ms() {
  const double* sums;
  long timed;
  if (h_) {
    sums = h_->sums, timed = h_->timed;
  } else {
    Impl_& I = *p_;
    sync();
    for (int i = 0; i < kRing; ++i) I.fold(i);
    sums = I.sums, timed = I.timed;
  }
  std::vector<std::pair<std::string, double>> v;
  for (int i = 0; i < 5; ++i) v.push_back({kPhase[i], timed ? sums[i] / timed : 0.0});
  v.push_back({"compute", v[1].second + v[2].second + v[3].second});
  return v;
}

void V5Runtime::reset_phases() {
  if (h_) {
    std::fill(std::begin(h_->sums), std::end(h_->sums), 0.0);
    h_->timed = 0;
    return;
  }
  Impl_& I = *p_;
  sync();
  std::fill(I.pending.begin(), I.pending.end(), false);
  std::fill(std::begin(I.sums), std::end(I.sums), 0.0);
  I.timed = 0;
}

std::string V5Runtime::describe_json() const {
  const Transport& X = h_ ? *h_->x : *p_->x;
  const Decomp mode = h_ ? h_->o.mode : p_->o.mode;
  const int dev = h_ ? -1 : p_->dev, nl = h_ ? 1 : p_->nl;
  const bool local = h_ ? h_->local : p_->local, lane = h_ ? h_->lane_path : p_->lane_path;
  const PlanStats s = stats();
  char b[1024];
  std::snprintf(b, sizeof b,
                "{\"transport\": \"%s\", \"ordering\": \"%s\", \"pipeline\": %s, \"chunks\": %d, \"groups\": %d, "
                "\"row_ways\": %d, \"out_rows_max\": %g, \"out_rows_mean\": %.4f, \"imbalance\": %.4f, "
                "\"conv1_redundancy\": %.4f, \"images_per_rank_max\": %g, \"transfers_per_step\": %zu, "
                "\"decomp\": \"%s\", \"device\": %d, \"input_source\": \"%s\", \"lanes\": %d, "
                "\"lane_path\": %s, \"input_placement_bytes\": %.0f, ",
                X.name(), X.ordering(), pipeline_ ? "true" : "false", lay_.chunks, s.groups, s.row_ways, s.rows_max,
                s.rows_mean, s.imbalance, s.conv1_redundancy, s.images_max, lay_.step_transfers().size(),
                mode == Decomp::PerLayer ? "per_layer" : "overlap", dev, local ? "local" : "root", nl,
                lane ? "true" : "false", lay_.input_placement_bytes());
  // bytes per step by phase: per rank (arrays over ranks) and the root's / busiest rank's totals
  const std::vector<RankBytes> rb = lay_.rank_bytes();
  std::string j = b;
  // whether this layout exchanges pool1 halos at all: the cost model's default may pick a pure batch
  // split (whole images per rank), which is V5 without its per-layer halo exchange; say so explicitly
  //  instead of leaving it to row_ways
  const size_t nhalo = lay_.sched.phase[static_cast<int>(Phase::P1Halo)].size();
  double halo_bytes = 0;
  for (const RankBytes& x : rb) halo_bytes += x.halo_sent;
  char h[160];
  std::snprintf(h, sizeof h, "\"halo_exchange\": \"%s\", \"halo_transfers_per_step\": %zu, \"halo_bytes_per_step\": %.0f, ",
                nhalo ? "pool1 rows between row-group neighbours" : "none (batch split: every rank whole images)", nhalo,
                halo_bytes);
  j += h;
  std::string imgs = "\"images_per_rank\": [";  // the plan's per-rank batch share (root shedding: rank 0's differs)
  for (int r = 0; r < lay_.plan.np; ++r) {
    const TilePlan& t = lay_.plan.tile(r);
    imgs += (r ? ", " : "") + std::to_string(t.out.empty() ? 0 : lay_.plan.images[lay_.plan.group_of[r]].size());
  }
  j += imgs + "], ";
  auto arr = [&](const char* name, double RankBytes::*f) {
    std::string a = "\"" + std::string(name) + "\": [";
    char t[32];
    for (size_t r = 0; r < rb.size(); ++r) {
      std::snprintf(t, sizeof t, "%s%.0f", r ? ", " : "", rb[r].*f);
      a += t;
    }
    return a + "]";
  };
  j += "\"bytes_per_step\": {" + arr("scatter_recv", &RankBytes::scatter_recv) + ", " +
       arr("scatter_sent", &RankBytes::scatter_sent) + ", " + arr("halo_sent", &RankBytes::halo_sent) + ", " +
       arr("halo_recv", &RankBytes::halo_recv) + ", " + arr("gather_sent", &RankBytes::gather_sent) + ", " +
       arr("gather_recv", &RankBytes::gather_recv) + "}}";
  return j;
}

}  // namespace anx
