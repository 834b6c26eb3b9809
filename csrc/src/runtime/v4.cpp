// V4 runtime: chunked, per-rank DMA from a shared pinned host segment (anx/v4.hpp).
#include "anx/v4.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "anx/trace.hpp"
#include "anx/cost.hpp"
#include "anx/v5.hpp"  // plan_stats

namespace anx {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("v4 ") + what + ": " + hipGetErrorString(e));
}
constexpr int kRing = 32;
constexpr int kMaxChunks = 16;
}  // namespace

struct V4Runtime::Impl_ {
  HostComm& c;
  RankInfo ri;
  V4Options o;
  BlocksDims d;
  HybridPlan plan;
  int rank = 0, np = 1, dev = 0, C = 1, n = 0;
  TilePlan t;
  RowRange im;
  std::unique_ptr<BlocksEngine> eng;
  // shared segment
  std::string shm_name;
  char* seg = nullptr;
  size_t seg_bytes = 0, in_bytes = 0, out_bytes = 0;
  bool registered = false;
  size_t in_row = 0, out_row = 0;  // bytes
  size_t tin_img = 0, tout_img = 0;  // bytes of one image's tile rows (input / output)
  float* d_in[2] = {nullptr, nullptr};
  float* d_y[2] = {nullptr, nullptr};
  std::vector<int> lo;
  hipStream_t sh = nullptr, st = nullptr, sd = nullptr;
  std::vector<hipEvent_t> e_in[2], e_cmp[2], e_out[2];
  long k = 0;
  std::vector<std::vector<hipEvent_t>> ring;
  std::vector<bool> pending;
  int ring_pos = 0;
  double sums[3] = {0, 0, 0};
  long timed = 0;

  bool created = false;  // rank 0 created the segment name and has not unlinked it yet

  Impl_(HostComm& cc, const RankInfo& r, const V4Options& oo) : c(cc), ri(r), o(oo) {}
  // Frees whatever the constructor got to (it may have thrown half way): engine, device buffers,
  // events, streams, the pinned registration, the mapping and (rank 0, before the others opened it)
  // the segment name.
  ~Impl_() {
    eng.reset();
    for (int p = 0; p < 2; ++p) {
      if (d_in[p]) (void)hipFree(d_in[p]);
      if (d_y[p]) (void)hipFree(d_y[p]);
      for (auto* v : {&e_in[p], &e_cmp[p], &e_out[p]})
        for (hipEvent_t e : *v) (void)hipEventDestroy(e);
    }
    for (auto& e : ring)
      for (hipEvent_t v : e) (void)hipEventDestroy(v);
    for (hipStream_t s : {sh, st, sd})
      if (s) (void)hipStreamDestroy(s);
    if (registered) (void)hipHostUnregister(seg);
    if (seg) munmap(seg, seg_bytes);
    if (created) shm_unlink(shm_name.c_str());
  }
  hipEvent_t event(bool timing = false) {
    hipEvent_t e = nullptr;
    hip_ok(hipEventCreateWithFlags(&e, timing ? hipEventDefault : hipEventDisableTiming), "hipEventCreate");
    return e;
  }
  void fold(int i) {
    if (!pending[i]) return;
    auto& e = ring[i];
    hip_ok(hipEventSynchronize(e[4]), "hipEventSynchronize");
    auto ms = [&](int a, int b) {
      float v = 0;
      hip_ok(hipEventElapsedTime(&v, e[a], e[b]), "hipEventElapsedTime");
      return static_cast<double>(v);
    };
    sums[0] += ms(0, 1);
    sums[1] += ms(2, 3);
    sums[2] += ms(3, 4);
    ++timed;
    pending[i] = false;
  }
  char* in_at(int img) const { return seg + static_cast<size_t>(img) * d.H * in_row; }
  char* out_at(int img) const { return seg + in_bytes + static_cast<size_t>(img) * d.Hp2 * out_row; }
};

V4Runtime::V4Runtime(HostComm& c, const RankInfo& ri, const BlockSpec& b1, const BlockSpec& b2, int H, int W,
                     const HostWeights& w, const V4Options& o)
    : p_(std::make_unique<Impl_>(c, ri, o)) {
  Impl_& I = *p_;
  I.rank = c.rank();
  I.np = c.size();
  I.d = blocks_dims(H, W, b1, b2);
  if (ri.nnodes > 1) throw std::runtime_error("v4 shared host staging is single-node (one host segment)");
  // default split: the cost model's (anx/cost.hpp): V4 is H2D-bound, so the batch split wins whenever
  // every rank gets whole images (a row split adds the rows' receptive-field overlap to each H2D)
  const int rw = o.row_ways < 0 ? pick_row_ways(Workload::V4, I.np, o.batch, InputSource::Root, Decomp::Overlap,
                                                cost_params(o.cost), b1, b2, H, W)
                                : o.row_ways;
  if (!make_hybrid_plan(H, W, I.np, o.batch, rw, Decomp::Overlap, I.plan, b1, b2))
    throw std::runtime_error("v4: invalid plan");
  I.t = I.plan.tile(I.rank);
  I.im = I.plan.images[I.plan.group_of[I.rank]];
  I.n = I.t.out.empty() ? 0 : I.im.size();
  int min_n = 1 << 30;
  for (int q = 0; q < I.np; ++q)
    if (!I.plan.tile(q).out.empty() && !I.plan.images[I.plan.group_of[q]].empty())
      min_n = std::min(min_n, I.plan.images[I.plan.group_of[q]].size());
  // auto: 4 chunks of >= 16 images (the first H2D and the last D2H are the exposed ends; 256 images at
  // N=1: 4 chunks 87.2k img/s, 8: 82.7k, 16: 75.2k, profiles/r03_v4_chunks.jsonl)
  I.C = std::max(1, std::min({o.chunks > 0 ? o.chunks : std::max(1, std::min(4, min_n / 16)), min_n, kMaxChunks}));
  for (int cc = 0; cc <= I.C; ++cc) I.lo.push_back(I.n * cc / I.C);

  // weights (host broadcast: V4 stages through the host by definition)
  HostWeights hw;
  init_const(hw, b1, b2);
  if (I.rank == 0) hw = w;
  for (auto* v : {&hw.w1, &hw.b1, &hw.w2, &hw.b2}) c.bcast(v->data(), v->size() * 4, 0);

  int ndev = 0;
  hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  if (ndev < 1) throw std::runtime_error("v4 needs a GPU");
  I.dev = ri.local_rank % ndev;
  hip_ok(hipSetDevice(I.dev), "hipSetDevice");

  // the shared segment: created by rank 0, mapped by everyone, unlinked once all have it open
  I.in_row = static_cast<size_t>(W) * I.d.C0 * 4;
  I.out_row = static_cast<size_t>(I.d.Wp2) * I.d.C2 * 4;
  I.in_bytes = static_cast<size_t>(o.batch) * H * I.in_row;
  I.out_bytes = static_cast<size_t>(o.batch) * I.d.Hp2 * I.out_row;
  I.seg_bytes = I.in_bytes + I.out_bytes;
  char name[96];
  std::snprintf(name, sizeof name, "/anx_v4_%d_%d", ri.master_port, static_cast<int>(getpid()));
  if (I.rank == 0) I.shm_name = name;
  char nb[96] = {0};
  std::snprintf(nb, sizeof nb, "%s", I.shm_name.c_str());
  c.bcast(nb, sizeof nb, 0);
  I.shm_name = nb;
  struct Fd {  // closes the descriptor on every path out of here
    int v = -1;
    ~Fd() {
      if (v >= 0) close(v);
    }
  } fd;
  if (I.rank == 0) {
    fd.v = shm_open(I.shm_name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd.v >= 0) I.created = true;
    if (fd.v < 0 || ftruncate(fd.v, static_cast<off_t>(I.seg_bytes)) != 0)
      throw std::runtime_error("v4: cannot create shared segment " + I.shm_name + ": " + std::strerror(errno));
  }
  c.barrier();
  if (I.rank != 0) fd.v = shm_open(I.shm_name.c_str(), O_RDWR, 0600);
  if (fd.v < 0) throw std::runtime_error("v4: cannot open shared segment " + I.shm_name + ": " + std::strerror(errno));
  void* m = mmap(nullptr, I.seg_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd.v, 0);
  if (m == MAP_FAILED) throw std::runtime_error(std::string("v4: mmap: ") + std::strerror(errno));
  I.seg = static_cast<char*>(m);
  c.barrier();
  if (I.rank == 0) {
    shm_unlink(I.shm_name.c_str());
    I.created = false;
  }
  hip_ok(hipHostRegister(I.seg, I.seg_bytes, hipHostRegisterDefault), "hipHostRegister");
  I.registered = true;

  I.eng = std::make_unique<BlocksEngine>(b1, b2, H, W, hw, std::max(1, I.n), o.impl, o.knobs);
  I.tin_img = static_cast<size_t>(I.t.in.size()) * I.in_row;
  I.tout_img = static_cast<size_t>(I.t.out.size()) * I.out_row;
  for (int p = 0; p < 2; ++p) {
    hip_ok(hipMalloc(&I.d_in[p], std::max<size_t>(4, I.n * I.tin_img)), "hipMalloc");
    hip_ok(hipMalloc(&I.d_y[p], std::max<size_t>(4, I.n * I.tout_img)), "hipMalloc");
    for (int cc = 0; cc < I.C; ++cc) {
      I.e_in[p].push_back(I.event());
      I.e_cmp[p].push_back(I.event());
      I.e_out[p].push_back(I.event());
    }
  }
  hip_ok(hipStreamCreateWithFlags(&I.sh, hipStreamNonBlocking), "hipStreamCreate");
  hip_ok(hipStreamCreateWithFlags(&I.st, hipStreamNonBlocking), "hipStreamCreate");
  hip_ok(hipStreamCreateWithFlags(&I.sd, hipStreamNonBlocking), "hipStreamCreate");
  I.ring.resize(kRing);
  for (auto& e : I.ring)
    for (int i = 0; i < 5; ++i) e.push_back(I.event(true));
  I.pending.assign(kRing, false);
  c.barrier();
}

V4Runtime::~V4Runtime() {
  if (!p_) return;
  (void)hipDeviceSynchronize();
  try {
    p_->c.barrier();  // every rank's copies out of / into the segment are done
  } catch (...) {
  }
  p_.reset();  // Impl_'s destructor frees everything
}

float* V4Runtime::host_input() const { return reinterpret_cast<float*>(p_->seg); }
const float* V4Runtime::host_output() const { return reinterpret_cast<const float*>(p_->seg + p_->in_bytes); }
int V4Runtime::chunks() const { return p_->C; }
const HybridPlan& V4Runtime::plan() const { return p_->plan; }
size_t V4Runtime::h2d_bytes_per_step() const { return p_->n * p_->tin_img; }
size_t V4Runtime::d2h_bytes_per_step() const { return p_->n * p_->tout_img; }

double V4Runtime::probe_h2d_gbps(int reps) {
  Impl_& I = *p_;
  sync();
  if (!I.n) return 0;
  hipEvent_t a = I.event(true), b = I.event(true);
  auto copy = [&] {
    hip_ok(hipMemcpy2DAsync(I.d_in[0], I.tin_img, I.in_at(I.im.lo) + I.t.in.lo * I.in_row,
                            static_cast<size_t>(I.d.H) * I.in_row, I.tin_img, I.n, hipMemcpyHostToDevice, I.sh),
           "H2D probe");
  };
  copy();  // first touch
  hip_ok(hipEventRecord(a, I.sh), "hipEventRecord");
  for (int i = 0; i < reps; ++i) copy();
  hip_ok(hipEventRecord(b, I.sh), "hipEventRecord");
  hip_ok(hipEventSynchronize(b), "hipEventSynchronize");
  float ms = 0;
  hip_ok(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime");
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return static_cast<double>(h2d_bytes_per_step()) * reps / (ms * 1e6);
}

void V4Runtime::input_ready() {
  sync();
  p_->c.barrier();
}

void V4Runtime::sync() {
  for (hipStream_t s : {p_->sh, p_->st, p_->sd}) hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
}

void V4Runtime::sync_all() {
  sync();
  p_->c.barrier();
}

void V4Runtime::step() {
  Impl_& I = *p_;
  const int par = static_cast<int>(I.k & 1);
  const int slot = I.ring_pos;
  I.fold(slot);
  auto& e = I.ring[slot];
  I.ring_pos = (I.ring_pos + 1) % kRing;
  auto wait = [](hipStream_t s, hipEvent_t ev) { hip_ok(hipStreamWaitEvent(s, ev, 0), "hipStreamWaitEvent"); };
  auto rec = [](hipEvent_t ev, hipStream_t s) { hip_ok(hipEventRecord(ev, s), "hipEventRecord"); };
  char* din = reinterpret_cast<char*>(I.d_in[par]);
  char* dy = reinterpret_cast<char*>(I.d_y[par]);
  rec(e[0], I.sh);
  for (int cc = 0; cc < I.C; ++cc) {  // H2D: this rank's images x tile rows, straight from the segment
    const int a = I.lo[cc], b = I.lo[cc + 1];
    if (b <= a) continue;
    wait(I.sh, I.e_cmp[par][cc]);  // step k-2's tile on this parity's chunk has read its input
    RoctxRange r("v4 h2d");
    hip_ok(hipMemcpy2DAsync(din + a * I.tin_img, I.tin_img, I.in_at(I.im.lo + a) + I.t.in.lo * I.in_row,
                            static_cast<size_t>(I.d.H) * I.in_row, I.tin_img, b - a, hipMemcpyHostToDevice, I.sh),
           "H2D");
    rec(I.e_in[par][cc], I.sh);
  }
  rec(e[1], I.sh);
  rec(e[2], I.st);
  for (int cc = 0; cc < I.C; ++cc) {
    const int a = I.lo[cc], b = I.lo[cc + 1];
    if (b <= a) continue;
    wait(I.st, I.e_in[par][cc]);
    wait(I.st, I.e_out[par][cc]);  // step k-2's D2H of this parity's chunk has read its output
    RoctxRange r("v4 tile");
    hip_ok(I.eng->tile_forward(reinterpret_cast<float*>(din + a * I.tin_img), b - a, I.t,
                               reinterpret_cast<float*>(dy + a * I.tout_img), I.st),
           "tile_forward");
    rec(I.e_cmp[par][cc], I.st);
  }
  rec(e[3], I.st);
  for (int cc = 0; cc < I.C; ++cc) {  // D2H: output rows straight into the segment
    const int a = I.lo[cc], b = I.lo[cc + 1];
    if (b <= a) continue;
    wait(I.sd, I.e_cmp[par][cc]);
    RoctxRange r("v4 d2h");
    hip_ok(hipMemcpy2DAsync(I.out_at(I.im.lo + a) + I.t.out.lo * I.out_row, static_cast<size_t>(I.d.Hp2) * I.out_row,
                            dy + a * I.tout_img, I.tout_img, I.tout_img, b - a, hipMemcpyDeviceToHost, I.sd),
           "D2H");
    rec(I.e_out[par][cc], I.sd);
  }
  rec(e[4], I.sd);
  I.pending[slot] = true;
  ++I.k;
}

std::vector<std::pair<std::string, double>> V4Runtime::phase_ms() {
  Impl_& I = *p_;
  sync();
  for (int i = 0; i < kRing; ++i) I.fold(i);
  const char* names[3] = {"h2d", "compute", "d2h"};
  std::vector<std::pair<std::string, double>> v;
  for (int i = 0; i < 3; ++i) v.push_back({names[i], I.timed ? I.sums[i] / I.timed : 0.0});
  return v;
}

void V4Runtime::reset_phases() {
  Impl_& I = *p_;
  sync();
  std::fill(I.pending.begin(), I.pending.end(), false);
  std::fill(std::begin(I.sums), std::end(I.sums), 0.0);
  I.timed = 0;
}

std::string V4Runtime::describe_json() const {
  const Impl_& I = *p_;
  const PlanStats s = plan_stats(I.plan);
  char b[900];
  // V4's halo is in its input: a row group's ranks each DMA their output rows' receptive field (overlap
  // tiles), so no exchange runs mid-network; with one row way (the cost model's usual pick) there is no
  // halo at all. Said explicitly, as V5's describe does.
  std::snprintf(b, sizeof b,
                "{\"staging\": \"shared pinned host segment, per-rank DMA\", \"chunks\": %d, \"groups\": %d, "
                "\"row_ways\": %d, \"imbalance\": %.4f, \"conv1_redundancy\": %.4f, \"images_per_rank_max\": %g, "
                "\"h2d_bytes_per_step_rank\": %zu, \"d2h_bytes_per_step_rank\": %zu, \"device\": %d, "
                "\"halo_exchange\": \"%s\"}",
                I.C, s.groups, s.row_ways, s.imbalance, s.conv1_redundancy, s.images_max, h2d_bytes_per_step(),
                d2h_bytes_per_step(), I.dev,
                s.row_ways > 1 ? "input halo rows in each rank's H2D (overlap tiles: no mid-network exchange)"
                               : "none (batch split: every rank whole images)");
  return b;
}

}  // namespace anx
