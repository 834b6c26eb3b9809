// V5 runtime: device-resident scatter -> stage1 -> chunked pool1 halos -> stage2 -> gather (anx/v5.hpp).
#include "anx/v5.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "anx/trace.hpp"

namespace anx {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("v5 ") + what + ": " + hipGetErrorString(e));
}
constexpr int kB = static_cast<int>(BufId::kCount);
constexpr int kMaxChunks = 16;  // the peer transport's halo channels
constexpr int kRing = 32;       // per-step timing event sets kept before they are folded in
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

int balanced_row_ways(int np, int batch, int H, int W) {
  if (np <= 1) return 1;
  int best = np;
  double best_imb = 1e30;
  for (int r = 2; r <= np; ++r) {
    if (np % r) continue;
    HybridPlan hp;
    if (!make_hybrid_plan(H, W, np, batch, r, Decomp::PerLayer, hp)) continue;
    const double imb = plan_stats(hp).imbalance;
    if (imb <= 1.1) return r;
    if (imb < best_imb - 1e-9) best_imb = imb, best = r;
  }
  return best;
}

std::string pick_v5_transport(const std::string& want, const RankInfo& ri, int ndev, bool dry) {
  const bool shared = !dry && ri.local_world > ndev;  // ranks of this node outnumber its GPUs
  const std::string tr = want == "auto" ? (shared && ri.nnodes == 1 ? "peer" : "rccl") : want;
  if (tr != "rccl" && tr != "peer") throw std::runtime_error("--transport must be auto, rccl or peer");
  if (tr == "peer" && ri.nnodes > 1)
    throw std::runtime_error("the peer transport (IPC) is single-node: use --transport rccl across nodes");
  if (tr == "rccl" && shared)
    throw std::runtime_error("v5 over RCCL needs one GPU per rank on each node (" + std::to_string(ri.local_world) +
                             " ranks, " + std::to_string(ndev) + " GPUs here; --transport peer shares a GPU)");
  return tr;
}

V5Layout make_v5_layout(int np, const BlockSpec& b1, const BlockSpec& b2, int H, int W, const V5Options& o) {
  V5Layout L;
  L.row_ways = o.row_ways < 0 ? balanced_row_ways(np, o.batch, H, W) : o.row_ways;
  if (!make_hybrid_plan(H, W, np, o.batch, L.row_ways, o.mode, L.plan, b1, b2))
    throw std::runtime_error("v5: invalid plan (row_ways " + std::to_string(L.row_ways) + " over " +
                             std::to_string(np) + " ranks)");
  const BlocksDims d = blocks_dims(H, W, b1, b2);
  const size_t in_row = static_cast<size_t>(d.W) * d.C0 * 4, out_row = static_cast<size_t>(d.Wp2) * d.C2 * 4;
  const size_t win_row = static_cast<size_t>(d.Wp1 + 2 * b2.conv.P) * d.C1 * 4;
  L.sched = make_step_schedule(L.plan, {in_row, out_row, win_row, d.H, d.Hp2});
  const auto& halos = L.sched.phase[static_cast<int>(Phase::P1Halo)];
  int min_imgs = 1 << 30;
  for (const Transfer& x : halos) min_imgs = std::min(min_imgs, static_cast<int>(x.height));
  // auto: chunks of >= 128 images, at most 4 (halo c moves while stage1 computes c+1; smaller launches
  // lose more to wave quantization than the exposed halo costs: profiles/r03_v5_halo.log)
  const int auto_chunks = std::max(1, std::min(4, min_imgs / 128));
  L.chunks = halos.empty() ? 1 : std::max(1, std::min({o.chunks > 0 ? o.chunks : auto_chunks, min_imgs, kMaxChunks}));
  for (int c = 0; c < L.chunks; ++c) L.halo_chunks.push_back(chunk_of(halos, c, L.chunks));
  return L;
}

std::vector<Transfer> V5Layout::step_transfers() const {
  std::vector<Transfer> v = sched.phase[static_cast<int>(Phase::Scatter)];
  for (const auto& c : halo_chunks) v.insert(v.end(), c.begin(), c.end());
  const auto& g = sched.phase[static_cast<int>(Phase::Gather)];
  v.insert(v.end(), g.begin(), g.end());
  return v;
}

std::vector<std::string> v5_dry_schedule(int rank, int np, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
                                         const V5Options& o, const std::string& transport) {
  const V5Layout L = make_v5_layout(np, b1, b2, H, W, o);
  std::unique_ptr<Transport> x =
      transport == "rccl" ? make_rccl_transport(nullptr, 0, rank) : make_peer_transport(nullptr, 0, rank, o.peer_sync);
  x->record_only = true;
  void* none[2][kB] = {};
  x->bind(L.sched, none, nullptr);
  x->run_phase(Phase::Scatter, L.sched.phase[0], nullptr, 0);
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
  std::vector<int> lo;  // this rank's chunk bounds (C + 1)
  size_t x_bytes = 0, yfull_bytes = 0, tile_bytes = 0, y_bytes = 0;
  float* d_x = nullptr;
  float* d_tile[2] = {nullptr, nullptr};
  float* d_y[2] = {nullptr, nullptr};
  float* d_yfull[2] = {nullptr, nullptr};
  bool alias_tile = false, alias_y = false;
  std::vector<float*> owned;  // device allocations to free
  hipStream_t st = nullptr, io = nullptr, hs = nullptr;
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
        if (o.poison && !alias_tile) {
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
      if (per_layer) {
        hip_ok(eng->stage2(n, t, d_y[par], st, lo[cc], lo[cc + 1]), "stage2");
        if (o.poison)  // the halo rows this rank received: the next step must bring them again
          for (const Transfer& h : L.halo_chunks[cc])
            if (h.dst == rank && h.src != rank)
              hip_ok(hipMemset2DAsync(reinterpret_cast<char*>(eng->q2_row_ptr(t, 0, t.q.lo)) + h.to.off, h.to.pitch,
                                      0xff, h.width, h.height, st),
                     "poison window");
      } else {
        hip_ok(eng->tile_forward(d_tile[par], n, t, d_y[par], st), "tile_forward");
        if (o.poison && !alias_tile) hip_ok(hipMemsetAsync(d_tile[par], 0xff, tile_bytes, st), "poison tile");
      }
    }
    rec(e[3 + 2 * C], st);
  }
};

V5Runtime::V5Runtime(HostComm& c, const RankInfo& ri, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
                     const HostWeights& w, const V5Options& o)
    : lay_(make_v5_layout(c.size(), b1, b2, H, W, o)) {
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
  I.x = I.tr == "rccl" ? make_rccl_transport(&c, I.dev, I.rank) : make_peer_transport(&c, I.dev, I.rank, o.peer_sync);
  pipeline_ = I.pipeline = o.pipeline < 0 ? I.tr == "rccl" : o.pipeline > 0;

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
  I.eng = std::make_unique<BlocksEngine>(b1, b2, H, W, hw, std::max(1, I.n), o.impl, o.knobs);
  hip_ok(hipStreamCreateWithFlags(&I.st, hipStreamNonBlocking), "hipStreamCreate");
  hip_ok(hipStreamCreateWithFlags(&I.io, hipStreamNonBlocking), "hipStreamCreate");
  hip_ok(hipStreamCreateWithFlags(&I.hs, hipStreamNonBlocking), "hipStreamCreate");

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
  if (I.n && o.mode == Decomp::PerLayer) {
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
  for (int p = 0; p < 2; ++p) I.e_sc[p] = I.event(), I.e_s2[p] = I.event();
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
  (void)hipDeviceSynchronize();
  try {
    I.c.barrier();  // nobody pushes into a peer's buffers any more
    I.x->close();   // collective: unmap, barrier, free own
  } catch (...) {
  }
  I.x.reset();
  I.eng.reset();
  for (float* p : I.owned) (void)hipFree(p);
  for (auto& e : I.ring)
    for (hipEvent_t v : e) (void)hipEventDestroy(v);
  for (hipEvent_t v : I.e_s1) (void)hipEventDestroy(v);
  for (hipEvent_t v : I.e_h) (void)hipEventDestroy(v);
  for (hipEvent_t v : {I.e_sc[0], I.e_sc[1], I.e_s2[0], I.e_s2[1], I.e_hdone})
    if (v) (void)hipEventDestroy(v);
  for (hipStream_t s : {I.st, I.io, I.hs})
    if (s) (void)hipStreamDestroy(s);
}

const char* V5Runtime::transport() const { return p_->x->name(); }
long V5Runtime::steps() const { return p_->k; }

void V5Runtime::set_input(const float* host_x) {
  Impl_& I = *p_;
  sync();
  if (I.rank == 0) {
    if (!host_x) throw std::runtime_error("v5 set_input: the root needs the batch");
    hip_ok(hipMemcpy(I.d_x, host_x, I.x_bytes, hipMemcpyHostToDevice), "H2D input");
  }
  I.prefetched = false;  // every rank drops its prefetched scatter: the next step scatters again
  I.c.barrier();
}

void V5Runtime::step() {
  Impl_& I = *p_;
  const long k = I.k;
  const int par = static_cast<int>(k & 1);
  const int slot = I.ring_pos;
  I.fold(slot);
  std::vector<hipEvent_t>& e = I.ring[slot];
  I.ring_pos = (I.ring_pos + 1) % kRing;
  if (!I.pipeline) {  // every phase on the compute stream
    I.rec(e[0], I.st);
    I.scatter(k, I.st);
    I.rec(e[1], I.st);
    I.compute(k, e);
    I.gather(k, I.st);
    I.rec(e.back(), I.st);
  } else {
    // io runs scatter(k+1) while st computes step k, then gather(k) once stage2(k) is done; st starts
    // step k+1 as soon as scatter(k+1) has landed. Every rank issues the phases in the same order
    // (scatter k+1, gather k), as RCCL's in-order matching and the peer flag counters require.
    if (!I.prefetched) {
      I.scatter(k, I.io);
      I.rec(I.e_sc[par], I.io);
    }
    I.rec(e[0], I.st);
    I.wait(I.st, I.e_sc[par]);
    I.rec(e[1], I.st);
    I.compute(k, e);
    I.rec(I.e_s2[par], I.st);
    I.scatter(k + 1, I.io);
    I.rec(I.e_sc[par ^ 1], I.io);
    I.prefetched = true;
    I.wait(I.io, I.e_s2[par]);
    I.gather(k, I.io);
    I.rec(e.back(), I.io);
  }
  I.pending[slot] = true;
  ++I.k;
}

void V5Runtime::sync() {
  Impl_& I = *p_;
  for (hipStream_t s : {I.st, I.io, I.hs}) hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
}

void V5Runtime::output(float* host_y) {
  Impl_& I = *p_;
  sync();
  if (I.rank != 0) return;
  if (I.k == 0) throw std::runtime_error("v5 output: no step has run");
  hip_ok(hipMemcpy(host_y, I.d_yfull[(I.k - 1) & 1], I.yfull_bytes, hipMemcpyDeviceToHost), "D2H output");
}

std::vector<std::pair<std::string, double>> V5Runtime::phase_ms() {
  Impl_& I = *p_;
  sync();
  for (int i = 0; i < kRing; ++i) I.fold(i);
  std::vector<std::pair<std::string, double>> v;
  for (int i = 0; i < 5; ++i) v.push_back({kPhase[i], I.timed ? I.sums[i] / I.timed : 0.0});
  return v;
}

void V5Runtime::reset_phases() {
  Impl_& I = *p_;
  sync();
  std::fill(I.pending.begin(), I.pending.end(), false);
  std::fill(std::begin(I.sums), std::end(I.sums), 0.0);
  I.timed = 0;
}

std::string V5Runtime::describe_json() const {
  const Impl_& I = *p_;
  const PlanStats s = stats();
  char b[768];
  std::snprintf(b, sizeof b,
                "{\"transport\": \"%s\", \"ordering\": \"%s\", \"pipeline\": %s, \"chunks\": %d, \"groups\": %d, "
                "\"row_ways\": %d, \"out_rows_max\": %g, \"out_rows_mean\": %.4f, \"imbalance\": %.4f, "
                "\"conv1_redundancy\": %.4f, \"images_per_rank_max\": %g, \"transfers_per_step\": %zu, "
                "\"decomp\": \"%s\", \"device\": %d}",
                I.x->name(), I.x->ordering(),
                pipeline_ ? "true" : "false", lay_.chunks, s.groups, s.row_ways, s.rows_max, s.rows_mean, s.imbalance,
                s.conv1_redundancy, s.images_max, lay_.step_transfers().size(),
                I.o.mode == Decomp::PerLayer ? "per_layer" : "overlap", I.dev);
  return b;
}

}  // namespace anx
