// One-step transfer schedule and its transports (see anx/schedule.hpp).
#include "anx/schedule.hpp"

#include <rccl/rccl.h>

#include <array>
#include <cstdio>
#include <tuple>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>

namespace anx {

namespace {
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
const char* kBufName[] = {"X", "Tile", "Win", "Y", "YFull"};
constexpr int kB = static_cast<int>(BufId::kCount);
}  // namespace

const char* phase_name(Phase p) {
  switch (p) {
    case Phase::Scatter: return "scatter";
    case Phase::P1Halo: return "halo_p1";
    case Phase::Gather: return "gather";
  }
  return "?";
}

std::string Transfer::str() const {
  char b[200];
  std::snprintf(b, sizeof b, "%s %d->%d w=%zu h=%zu from=%s+%zu/%zu to=%s+%zu/%zu", phase_name(phase), src, dst, width,
                height, kBufName[static_cast<int>(from.buf)], from.off, from.pitch, kBufName[static_cast<int>(to.buf)],
                to.off, to.pitch);
  return b;
}

Schedule make_step_schedule(const HybridPlan& p, const StepGeometry& g) {
  Schedule s;
  s.np = p.np;
  auto& sc = s.phase[static_cast<int>(Phase::Scatter)];
  auto& ga = s.phase[static_cast<int>(Phase::Gather)];
  auto& ha = s.phase[static_cast<int>(Phase::P1Halo)];
  for (int q = 0; q < p.np; ++q) {
    const TilePlan& t = p.tile(q);
    const RowRange im = p.images[p.group_of[q]];
    if (t.out.empty() || im.empty()) continue;
    const size_t n = static_cast<size_t>(im.size());
    sc.push_back({Phase::Scatter, 0, q,
                  {BufId::X, (static_cast<size_t>(im.lo) * g.H + t.in.lo) * g.in_row, g.H * g.in_row},
                  {BufId::Tile, 0, t.in.size() * g.in_row}, t.in.size() * g.in_row, n});
    ga.push_back({Phase::Gather, q, 0, {BufId::Y, 0, t.out.size() * g.out_row},
                  {BufId::YFull, (static_cast<size_t>(im.lo) * g.Hp2 + t.out.lo) * g.out_row, g.Hp2 * g.out_row},
                  t.out.size() * g.out_row, n});
  }
  for (int grp = 0; grp < p.groups; ++grp) {
    const DecompPlan& rp = p.row_plans[grp];
    const int base = p.group_first[grp];
    const size_t n = static_cast<size_t>(p.images[grp].size());
    if (n == 0) continue;
    for (const HaloXfer& h : rp.p1_halos) {
      const TilePlan &ts = rp.tiles[h.src], &td = rp.tiles[h.dst];
      ha.push_back({Phase::P1Halo, base + h.src, base + h.dst,
                    {BufId::Win, (h.rows.lo - ts.q.lo) * g.win_row, ts.q.size() * g.win_row},
                    {BufId::Win, (h.rows.lo - td.q.lo) * g.win_row, td.q.size() * g.win_row},
                    h.rows.size() * g.win_row, n});
    }
  }
  return s;
}

namespace {

// Shared by the device transports: buffers per step parity, local 2-D copies.
struct DeviceBase : Transport {
  int rank_;
  void* buf_[2][kB] = {};
  char* at(int par, const Region& r) const { return static_cast<char*>(buf_[par][static_cast<int>(r.buf)]) + r.off; }
  void bind_bufs(void* const bufs[2][kB]) {
    for (int p = 0; p < 2; ++p)
      for (int b = 0; b < kB; ++b) buf_[p][b] = bufs[p][b];
  }
  void copy2d(char* dst, size_t dpitch, const char* src, size_t spitch, size_t w, size_t h, hipStream_t s) {
    hip_ok(hipMemcpy2DAsync(dst, dpitch, src, spitch, w, h, hipMemcpyDeviceToDevice, s), "hipMemcpy2DAsync");
  }
  // src == dst transfers (the root's own scatter / gather share) on the compute stream
  void local(const std::vector<Transfer>& xs, hipStream_t compute, int par) {
    for (const Transfer& x : xs)
      if (x.src == rank_ && x.dst == rank_) {
        note(x);
        if (!record_only) copy2d(at(par, x.to), x.to.pitch, at(par, x.from), x.from.pitch, x.width, x.height, compute);
      }
  }
};

// ---------------------------------------------------------------------------------------- RCCL
// Grouped ncclSend/ncclRecv on the communicator's stream, ordered after the compute stream by an
// event and before it by another: non-contiguous blocks are packed into / unpacked from staging
// buffers with one 2-D copy each (allocated once per transfer).
struct RcclTransport : DeviceBase {
  HostComm& hc_;
  int device_;
  std::unique_ptr<DeviceComm> dc_;
  std::map<std::pair<int, int>, void*> stage_;  // (phase, transfer index) -> contiguous staging
  RcclTransport(HostComm& c, int device, int rank) : hc_(c), device_(device) { rank_ = rank; }
  ~RcclTransport() override { close(); }
  const char* name() const override { return "rccl"; }
  void bind(const Schedule&, void* const bufs[2][kB], hipStream_t) override {
    bind_bufs(bufs);
    if (!record_only) dc_ = std::make_unique<DeviceComm>(hc_, device_);
  }
  void* staging(int ph, int i, size_t bytes) {
    void*& p = stage_[{ph, i}];
    if (!p) hip_ok(hipMalloc(&p, bytes), "hipMalloc staging");
    return p;
  }
  void run_phase(Phase ph, const std::vector<Transfer>& xs, hipStream_t compute, int par) override {
    local(xs, compute, par);
    bool any = false;
    for (const Transfer& x : xs) any |= (x.src != x.dst) && (x.src == rank_ || x.dst == rank_);
    if (!any) return;
    hipStream_t cs = record_only ? nullptr : dc_->stream();
    if (!record_only) dc_->after(compute);
    std::vector<std::pair<const Transfer*, void*>> unpack;
    // pack
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.src != rank_ || x.dst == rank_ || record_only || x.from.pitch == x.width) continue;
      copy2d(static_cast<char*>(staging(static_cast<int>(ph), static_cast<int>(i), x.bytes())), x.width,
             at(par, x.from), x.from.pitch, x.width, x.height, cs);
    }
    if (!record_only) dc_->group_start();
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.src == x.dst || (x.src != rank_ && x.dst != rank_)) continue;
      note(x);
      if (record_only) continue;
      if (x.src == rank_) {
        const void* src = x.from.pitch == x.width ? at(par, x.from)
                                                  : staging(static_cast<int>(ph), static_cast<int>(i), x.bytes());
        dc_->send(src, x.bytes(), x.dst);
      } else {
        void* dst = x.to.pitch == x.width ? static_cast<void*>(at(par, x.to))
                                          : staging(static_cast<int>(ph), static_cast<int>(i), x.bytes());
        if (x.to.pitch != x.width) unpack.push_back({&x, dst});
        dc_->recv(dst, x.bytes(), x.src);
      }
    }
    if (record_only) return;
    dc_->group_end();
    for (auto& u : unpack)
      copy2d(at(par, u.first->to), u.first->to.pitch, static_cast<char*>(u.second), u.first->width, u.first->width,
             u.first->height, cs);
    dc_->before(compute);
  }
  void end_step(hipStream_t) override {}  // receive buffers are reused in comm-stream order
  void close() override {
    for (auto& kv : stage_) (void)hipFree(kv.second);
    stage_.clear();
    dc_.reset();
  }
};

// ---------------------------------------------------------------------------------------- peer
// Every byte moves by ONE hipMemcpy2DAsync from the sender's buffer straight into the receiver's
// IPC-mapped buffer (Tile / YFull of the step's parity; a per-transfer parity staging slot for the
// conv2-window halos, unpacked by the receiver on its compute stream). Ordering without host stream
// syncs: the sender's copy stream waits for its compute stream (event), pushes, records its IPC
// event for (phase, parity) and posts a 4-byte "sent" note over the host channel; the receiver's
// host thread takes the note, and its compute stream waits for the sender's IPC event. Receive
// buffers alternate by step parity, so a push of step k+1 can never land in a buffer step k is
// still reading: the sender only gets to step k+1 of a phase after data of the receiver's step k
// (the root's scatter of step k+2 follows its gather of step k, which waits for every rank's
// stage2 of step k).
struct PeerTransport : DeviceBase {
  HostComm& c_;
  int device_;
  hipStream_t cs_ = nullptr;
  hipEvent_t ready_ = nullptr;
  hipEvent_t drained_ = nullptr;                 // end_step: all pushes issued so far are done
  hipEvent_t sent_[3][2] = {};                   // own IPC events (phase, parity)
  std::vector<std::array<std::array<hipEvent_t, 2>, 3>> peer_sent_;  // opened IPC events of every rank
  std::vector<std::array<void*, kB * 2>> peer_buf_;                  // mapped buffers of every rank
  std::map<std::tuple<int, int, int>, void*> halo_stage_;            // (src, transfer idx, parity) -> own slot
  std::vector<std::map<std::tuple<int, int, int>, void*>> peer_halo_; // mapped halo slots of every rank
  std::vector<void*> opened_;
  std::vector<hipEvent_t> opened_ev_;
  int np_ = 1;
  const Schedule* sched_ = nullptr;

  PeerTransport(HostComm& c, int device, int rank) : c_(c), device_(device) { rank_ = rank; }
  ~PeerTransport() override { close(); }
  const char* name() const override { return "peer"; }

  void* share(void* mine, int r) {  // collective: rank r's allocation mapped here
    hipIpcMemHandle_t h{};
    const int has = mine ? 1 : 0;
    int flag = has;
    if (r == rank_ && mine) hip_ok(hipIpcGetMemHandle(&h, mine), "hipIpcGetMemHandle");
    c_.bcast(&flag, sizeof flag, r);
    if (!flag) return nullptr;
    c_.bcast(&h, sizeof h, r);
    if (r == rank_) return mine;
    void* p = nullptr;
    hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened_.push_back(p);
    return p;
  }
  hipEvent_t share_ev(hipEvent_t mine, int r) {
    hipIpcEventHandle_t h{};
    if (r == rank_) hip_ok(hipIpcGetEventHandle(&h, mine), "hipIpcGetEventHandle");
    c_.bcast(&h, sizeof h, r);
    if (r == rank_) return mine;
    hipEvent_t e = nullptr;
    hip_ok(hipIpcOpenEventHandle(&e, h), "hipIpcOpenEventHandle");
    opened_ev_.push_back(e);
    return e;
  }

  void bind(const Schedule& sch, void* const bufs[2][kB], hipStream_t) override {
    sched_ = &sch;
    bind_bufs(bufs);
    np_ = c_.size();
    if (record_only) return;
    hip_ok(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking), "hipStreamCreate");
    hip_ok(hipEventCreateWithFlags(&ready_, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventCreateWithFlags(&drained_, hipEventDisableTiming), "hipEventCreate");
    for (auto& ph : sent_)
      for (auto& e : ph)
        hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventInterprocess), "hipEventCreate IPC");
    peer_buf_.assign(np_, {});
    peer_sent_.assign(np_, {});
    for (int r = 0; r < np_; ++r) {
      for (int p = 0; p < 2; ++p)
        for (int b = 0; b < kB; ++b) {
          // only buffers that are written remotely: Tile (scatter) and YFull (gather)
          const bool remote = b == static_cast<int>(BufId::Tile) || b == static_cast<int>(BufId::YFull);
          peer_buf_[r][p * kB + b] = remote ? share(r == rank_ ? buf_[p][b] : nullptr, r) : nullptr;
        }
      for (int ph = 0; ph < 3; ++ph)
        for (int p = 0; p < 2; ++p) peer_sent_[r][ph][p] = share_ev(sent_[ph][p], r);
    }
    // halo slots: the receiver owns one per incoming halo transfer and parity
    peer_halo_.assign(np_, {});
    const auto& hs = sched_->phase[static_cast<int>(Phase::P1Halo)];
    for (size_t i = 0; i < hs.size(); ++i)
      for (int p = 0; p < 2; ++p) {
        void* mine = nullptr;
        if (hs[i].dst == rank_) {
          hip_ok(hipMalloc(&mine, hs[i].bytes()), "hipMalloc halo slot");
          halo_stage_[{hs[i].src, static_cast<int>(i), p}] = mine;
        }
        peer_halo_[hs[i].src][{hs[i].dst, static_cast<int>(i), p}] = share(mine, hs[i].dst);
      }
  }

  void run_phase(Phase ph, const std::vector<Transfer>& xs, hipStream_t compute, int par) override {
    local(xs, compute, par);
    const int phi = static_cast<int>(ph);
    const bool halo = ph == Phase::P1Halo;
    bool sends = false;
    std::vector<int> notify;
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.src != rank_ || x.dst == rank_) continue;
      note(x);
      if (record_only) continue;
      if (!sends) {
        hip_ok(hipEventRecord(ready_, compute), "hipEventRecord");
        hip_ok(hipStreamWaitEvent(cs_, ready_, 0), "hipStreamWaitEvent");
        sends = true;
      }
      char* dst = halo ? static_cast<char*>(peer_halo_[rank_][{x.dst, static_cast<int>(i), par}])
                       : static_cast<char*>(peer_buf_[x.dst][par * kB + static_cast<int>(x.to.buf)]) + x.to.off;
      copy2d(dst, halo ? x.width : x.to.pitch, at(par, x.from), x.from.pitch, x.width, x.height, cs_);
      notify.push_back(x.dst);
    }
    if (sends) {
      hip_ok(hipEventRecord(sent_[phi][par], cs_), "hipEventRecord IPC");
      const int msg = phi * 2 + par;
      for (int d : notify) c_.isend(&msg, sizeof msg, d);
      c_.wait_all();
    }
    // receive: take each sender's note, then make the compute stream wait for its IPC event
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.dst != rank_ || x.src == rank_) continue;
      note(x);
      if (record_only) continue;
      int msg = -1;
      c_.recv(&msg, sizeof msg, x.src);
      if (msg != phi * 2 + par) throw std::runtime_error("peer transport: out-of-order note");
      hip_ok(hipStreamWaitEvent(compute, peer_sent_[x.src][phi][par], 0), "hipStreamWaitEvent IPC");
      if (halo)
        copy2d(at(par, x.to), x.to.pitch, static_cast<char*>(halo_stage_[{x.src, static_cast<int>(i), par}]), x.width,
               x.width, x.height, compute);
    }
  }
  // The stream waits for every push this rank has issued so far (its send buffers may be rewritten
  // after that; the receivers' buffers are ordered by their own IPC-event waits).
  void end_step(hipStream_t s) override {
    if (record_only || !cs_) return;
    hip_ok(hipEventRecord(drained_, cs_), "hipEventRecord");
    hip_ok(hipStreamWaitEvent(s, drained_, 0), "hipStreamWaitEvent");
  }
  void close() override {
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    for (hipEvent_t e : opened_ev_) (void)hipEventDestroy(e);
    opened_ev_.clear();
    for (auto& kv : halo_stage_) (void)hipFree(kv.second);
    halo_stage_.clear();
    for (auto& ph : sent_)
      for (auto& e : ph)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    if (ready_) (void)hipEventDestroy(ready_), ready_ = nullptr;
    if (drained_) (void)hipEventDestroy(drained_), drained_ = nullptr;
    if (cs_) (void)hipStreamDestroy(cs_), cs_ = nullptr;
  }
};

}  // namespace

std::unique_ptr<Transport> make_rccl_transport(HostComm& c, int device, int rank) {
  return std::make_unique<RcclTransport>(c, device, rank);
}
std::unique_ptr<Transport> make_peer_transport(HostComm& c, int device, int rank) {
  return std::make_unique<PeerTransport>(c, device, rank);
}

}  // namespace anx
