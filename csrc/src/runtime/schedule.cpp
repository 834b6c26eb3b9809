// One-step transfer schedule and its transports (see anx/schedule.hpp).
#include "anx/schedule.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <tuple>
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
  char b[220], ph[24];
  if (chunk >= 0) std::snprintf(ph, sizeof ph, "%s#%d", phase_name(phase), chunk);
  else std::snprintf(ph, sizeof ph, "%s", phase_name(phase));
  std::snprintf(b, sizeof b, "%s %d->%d w=%zu h=%zu from=%s+%zu/%zu to=%s+%zu/%zu", ph, src, dst, width, height,
                kBufName[static_cast<int>(from.buf)], from.off, from.pitch, kBufName[static_cast<int>(to.buf)], to.off,
                to.pitch);
  return b;
}

std::vector<Transfer> chunk_of(const std::vector<Transfer>& xs, int c, int chunks) {
  std::vector<Transfer> out;
  for (size_t i = 0; i < xs.size(); ++i) {
    const Transfer& x = xs[i];
    const size_t lo = x.height * c / chunks, hi = x.height * (c + 1) / chunks;
    if (hi <= lo) continue;
    Transfer y = x;
    y.chunk = c;
    y.seq = static_cast<int>(i);
    y.img0 = lo;
    y.from.off += lo * x.from.pitch;
    y.to.off += lo * x.to.pitch;
    y.height = hi - lo;
    out.push_back(y);
  }
  return out;
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
  // src == dst transfers (the root's own scatter / gather share) on the given stream; none when the
  // runtime aliased the two buffers (the root's whole-image tiles live inside X / YFull)
  void local(const std::vector<Transfer>& xs, hipStream_t compute, int par) {
    for (const Transfer& x : xs)
      if (x.src == rank_ && x.dst == rank_) {
        note(x);
        if (!record_only && at(par, x.to) != at(par, x.from))
          copy2d(at(par, x.to), x.to.pitch, at(par, x.from), x.from.pitch, x.width, x.height, compute);
      }
  }
  static bool remote(const Transfer& x, int r) { return x.src != x.dst && (x.src == r || x.dst == r); }
};

// ---------------------------------------------------------------------------------------- RCCL
// Grouped ncclSend/ncclRecv on a communicator stream, ordered after the given stream by an event and
// before it by another: non-contiguous blocks are packed into / unpacked from staging buffers with one
// 2-D copy each (allocated once per transfer and chunk). Two communicators: scatter / gather / weight
// broadcast on one, the pool1 halos on the other, so a halo chunk never queues behind the previous
// step's gather on one communicator stream.
// `loopback`: the same transport over the loopback DeviceComm (ranks sharing one GPU; anx/comm.hpp), so
// this code runs multi-rank on a one-GPU box exactly as it runs over RCCL. Ordering of the two
// communicators ("chain", the default): each phase's comm stream first waits for the other
// communicator's last queued op, so all device traffic of a rank is one total order, identical on
// every rank (phases are issued in the same order everywhere); no communicator can wait on a peer
// that is itself waiting behind the other one. "free" (ANX_V5_COMM_ORDER=free) lets them overlap.
struct RcclTransport : DeviceBase {
  HostComm* hc_;
  int device_;
  bool loopback_ = false, chain_ = true;
  std::unique_ptr<DeviceComm> dc_[2];
  DeviceComm* last_ = nullptr;  // communicator of the previous phase
  std::map<std::tuple<int, int, int>, void*> stage_;  // (phase, chunk, transfer) -> contiguous staging
  RcclTransport(HostComm* c, int device, int rank, bool loopback) : hc_(c), device_(device), loopback_(loopback) {
    rank_ = rank;
    const char* e = std::getenv("ANX_V5_COMM_ORDER");
    if (e && std::string(e) != "chain" && std::string(e) != "free")
      throw std::runtime_error("ANX_V5_COMM_ORDER must be chain or free");
    chain_ = !(e && std::string(e) == "free");
  }
  ~RcclTransport() override { close(); }
  const char* name() const override { return loopback_ ? "rccl-loopback" : "rccl"; }
  const char* ordering() const override { return chain_ ? "events, chained communicators" : "events"; }
  bool live() const { return !record_only && hc_ && hc_->size() > 1; }
  std::unique_ptr<DeviceComm> make_comm() {
    return loopback_ ? make_loopback_comm(*hc_, device_) : make_rccl_comm(*hc_, device_);
  }
  void connect() {
    if (live() && !dc_[0]) dc_[0] = make_comm();
  }
  void bcast(void* buf, size_t bytes, int root) override {
    if (!live()) return;
    connect();
    dc_[0]->bcast(buf, bytes, root);
    hip_ok(hipStreamSynchronize(dc_[0]->stream()), "hipStreamSynchronize");
  }
  void bind(const Schedule& s, void* const bufs[2][kB], hipStream_t) override {
    bind_bufs(bufs);
    if (!live()) return;
    connect();
    if (!s.phase[static_cast<int>(Phase::P1Halo)].empty()) dc_[1] = make_comm();
  }
  void* staging(Phase ph, const Transfer& x, size_t i) {
    void*& p = stage_[{static_cast<int>(ph), x.chunk, x.seq >= 0 ? x.seq : static_cast<int>(i)}];
    if (!p) hip_ok(hipMalloc(&p, x.bytes()), "hipMalloc staging");
    return p;
  }
  void run_phase(Phase ph, const std::vector<Transfer>& xs, hipStream_t compute, int par) override {
    local(xs, compute, par);
    bool any = false;
    for (const Transfer& x : xs) any |= remote(x, rank_);
    if (!any) return;
    DeviceComm* dc = record_only ? nullptr : dc_[ph == Phase::P1Halo && dc_[1] ? 1 : 0].get();
    hipStream_t cs = dc ? dc->stream() : nullptr;
    if (dc) {
      dc->after(compute);
      if (chain_ && last_) dc->after_comm(*last_);
      last_ = dc;
    }
    std::vector<std::pair<const Transfer*, void*>> unpack;
    for (size_t i = 0; i < xs.size(); ++i) {  // pack
      const Transfer& x = xs[i];
      if (x.src != rank_ || x.dst == rank_ || !dc || x.from.pitch == x.width) continue;
      copy2d(static_cast<char*>(staging(ph, x, i)), x.width, at(par, x.from), x.from.pitch, x.width, x.height, cs);
    }
    if (dc) dc->group_start();
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (!remote(x, rank_)) continue;
      note(x);
      if (!dc) continue;
      if (x.src == rank_) {
        dc->send(x.from.pitch == x.width ? at(par, x.from) : staging(ph, x, i), x.bytes(), x.dst);
      } else {
        void* dst = x.to.pitch == x.width ? static_cast<void*>(at(par, x.to)) : staging(ph, x, i);
        if (x.to.pitch != x.width) unpack.push_back({&x, dst});
        dc->recv(dst, x.bytes(), x.src);
      }
    }
    if (!dc) return;
    dc->group_end();
    for (auto& u : unpack)
      copy2d(at(par, u.first->to), u.first->to.pitch, static_cast<char*>(u.second), u.first->width, u.first->width,
             u.first->height, cs);
    dc->before(compute);
  }
  void close() override {
    for (auto& kv : stage_) (void)hipFree(kv.second);
    stage_.clear();
    last_ = nullptr;
    dc_[1].reset();
    dc_[0].reset();
  }
  void abort() override {
    for (auto& d : dc_)
      if (d) d->abort();
  }
};

// ---------------------------------------------------------------------------------------- peer
// Every byte moves by ONE hipMemcpy2DAsync from the sender's buffer straight into the receiver's
// IPC-mapped buffer (Tile / YFull of the step's parity; for the conv2-window halos a per-transfer,
// per-parity slot the receiver unpacks into its window on its own stream), issued on the stream the
// phase is given. Ordering, "flags" mode: every rank owns a word per (sender, channel) in device
// memory, IPC-mapped by the senders; after its pushes the sender's stream writes the next sequence
// number of that channel into the receiver's word (hipStreamWriteValue32: after every earlier command
// of the stream) and the receiver's stream waits for it (hipStreamWaitValue32 >=). Both sides count
// the same calls, so no host message is exchanged per phase. "notes" mode (fallback): IPC events per
// (channel, parity) plus a 4-byte host note over the TCP channel.
// Receive buffers alternate by step parity, so a push of step k+2 can only land after the receiver's
// step k consumed that parity: the root's scatter of step k+2 follows its gather of step k, which
// waits for every rank's stage2 of step k (anx/v5.hpp).
struct PeerTransport : DeviceBase {
  static constexpr int kMaxChunks = 16;
  static constexpr int kCh = 2 + kMaxChunks;  // scatter, gather, halo chunks
  HostComm* c_;
  int device_;
  bool flags_ = true;
  int np_ = 1;
  std::vector<std::array<void*, kB * 2>> peer_buf_;  // mapped Tile / YFull of every rank
  std::map<std::pair<int, int>, void*> slot_;        // own halo slots: (transfer, parity)
  std::map<std::pair<int, int>, void*> peer_slot_;   // receivers' slots this rank pushes into
  // flags mode
  uint32_t* flags_mine_ = nullptr;  // [np][kCh], written by the senders
  std::vector<uint32_t*> flags_of_;  // every rank's flag array, mapped
  std::vector<std::array<uint32_t, kCh>> sent_seq_, recv_seq_;
  // notes mode
  hipEvent_t sent_[kCh][2] = {};
  std::vector<std::array<std::array<hipEvent_t, 2>, kCh>> peer_sent_;
  std::vector<void*> opened_;
  std::vector<hipEvent_t> opened_ev_;
  bool connected_ = false;

  PeerTransport(HostComm* c, int device, int rank, const std::string& sync) : c_(c), device_(device) {
    rank_ = rank;
    std::string mode = sync;
    if (mode.empty()) {
      const char* e = std::getenv("ANX_PEER_SYNC");
      mode = e ? e : "flags";
    }
    if (mode != "flags" && mode != "notes") throw std::runtime_error("peer sync must be flags or notes");
    flags_ = mode == "flags";
  }
  ~PeerTransport() override { release(); }
  const char* name() const override { return "peer"; }
  const char* ordering() const override { return flags_ ? "flags" : "notes"; }
  static int channel(Phase ph, int chunk) {
    if (ph == Phase::Scatter) return 0;
    if (ph == Phase::Gather) return 1;
    if (chunk >= kMaxChunks) throw std::runtime_error("peer transport: too many halo chunks");
    return 2 + (chunk < 0 ? 0 : chunk);
  }

  void* share(void* mine, int r) {  // collective: rank r's allocation mapped here
    hipIpcMemHandle_t h{};
    int flag = mine ? 1 : 0;
    if (r == rank_ && mine) hip_ok(hipIpcGetMemHandle(&h, mine), "hipIpcGetMemHandle");
    c_->bcast(&flag, sizeof flag, r);
    if (!flag) return nullptr;
    c_->bcast(&h, sizeof h, r);
    if (r == rank_) return mine;
    void* p = nullptr;
    hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened_.push_back(p);
    return p;
  }
  hipEvent_t share_ev(hipEvent_t mine, int r) {
    hipIpcEventHandle_t h{};
    if (r == rank_) hip_ok(hipIpcGetEventHandle(&h, mine), "hipIpcGetEventHandle");
    c_->bcast(&h, sizeof h, r);
    if (r == rank_) return mine;
    hipEvent_t e = nullptr;
    hip_ok(hipIpcOpenEventHandle(&e, h), "hipIpcOpenEventHandle");
    opened_ev_.push_back(e);
    return e;
  }

  // collective: ordering primitives (flag words or IPC events) of every rank
  void connect() {
    if (connected_ || record_only) return;
    connected_ = true;
    np_ = c_->size();
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    if (flags_) {
      int can = 0;
      if (hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, device_) != hipSuccess || !can)
        throw std::runtime_error("peer transport: device lacks hipStreamWaitValue32 (set ANX_PEER_SYNC=notes)");
      const size_t bytes = static_cast<size_t>(np_) * kCh * sizeof(uint32_t);
      hip_ok(hipMalloc(reinterpret_cast<void**>(&flags_mine_), bytes), "hipMalloc flags");
      hip_ok(hipMemset(flags_mine_, 0, bytes), "hipMemset flags");
      hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
      flags_of_.assign(np_, nullptr);
      for (int r = 0; r < np_; ++r) flags_of_[r] = static_cast<uint32_t*>(share(r == rank_ ? flags_mine_ : nullptr, r));
      sent_seq_.assign(np_, {});
      recv_seq_.assign(np_, {});
    } else {
      for (auto& ch : sent_)
        for (auto& e : ch)
          hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventInterprocess), "hipEventCreate IPC");
      peer_sent_.assign(np_, {});
      for (int r = 0; r < np_; ++r)
        for (int ch = 0; ch < kCh; ++ch)
          for (int p = 0; p < 2; ++p) peer_sent_[r][ch][p] = share_ev(sent_[ch][p], r);
    }
  }

  void bcast(void* buf, size_t bytes, int root) override {
    if (record_only || !c_ || c_->size() == 1) return;
    connect();
    void* src = share(rank_ == root ? buf : nullptr, root);
    if (rank_ != root) hip_ok(hipMemcpy(buf, src, bytes, hipMemcpyDeviceToDevice), "hipMemcpy bcast");
    c_->barrier();  // every rank copied: unmap the root's buffer
    if (rank_ != root) {
      hip_ok(hipIpcCloseMemHandle(src), "hipIpcCloseMemHandle");
      opened_.pop_back();
    }
  }

  void bind(const Schedule& sch, void* const bufs[2][kB], hipStream_t) override {
    bind_bufs(bufs);
    if (record_only) return;
    connect();
    peer_buf_.assign(np_, {});
    for (int r = 0; r < np_; ++r)
      for (int p = 0; p < 2; ++p)
        for (BufId b : {BufId::Tile, BufId::YFull})  // the buffers written remotely
          peer_buf_[r][p * kB + static_cast<int>(b)] = share(r == rank_ ? buf_[p][static_cast<int>(b)] : nullptr, r);
    const auto& hs = sch.phase[static_cast<int>(Phase::P1Halo)];
    for (size_t i = 0; i < hs.size(); ++i)
      for (int p = 0; p < 2; ++p) {
        void* mine = nullptr;
        if (hs[i].dst == rank_) {
          hip_ok(hipMalloc(&mine, hs[i].bytes()), "hipMalloc halo slot");
          slot_[{static_cast<int>(i), p}] = mine;
        }
        void* m = share(mine, hs[i].dst);
        if (hs[i].src == rank_) peer_slot_[{static_cast<int>(i), p}] = m;
      }
  }

  void run_phase(Phase ph, const std::vector<Transfer>& xs, hipStream_t s, int par) override {
    local(xs, s, par);
    const bool halo = ph == Phase::P1Halo;
    std::vector<int> to;  // receivers of this rank's pushes, in first-push order
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.src != rank_ || x.dst == rank_) continue;
      note(x);
      if (record_only) continue;
      const int seq = x.seq >= 0 ? x.seq : static_cast<int>(i);
      char* dst = halo ? static_cast<char*>(peer_slot_.at({seq, par})) + x.img0 * x.width
                       : static_cast<char*>(peer_buf_[x.dst][par * kB + static_cast<int>(x.to.buf)]) + x.to.off;
      copy2d(dst, halo ? x.width : x.to.pitch, at(par, x.from), x.from.pitch, x.width, x.height, s);
      if (std::find(to.begin(), to.end(), x.dst) == to.end()) to.push_back(x.dst);
    }
    const int ch = xs.empty() ? 0 : channel(ph, xs.front().chunk);
    if (!to.empty()) {
      if (flags_) {
        for (int d : to)
          hip_ok(hipStreamWriteValue32(s, flags_of_[d] + rank_ * kCh + ch, ++sent_seq_[d][ch], 0),
                 "hipStreamWriteValue32");
      } else {
        hip_ok(hipEventRecord(sent_[ch][par], s), "hipEventRecord IPC");
        const int msg = ch * 2 + par;
        for (int d : to) c_->isend(&msg, sizeof msg, d);
        c_->wait_all();
      }
    }
    std::vector<int> from;
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.dst != rank_ || x.src == rank_) continue;
      note(x);
      if (record_only) continue;
      if (std::find(from.begin(), from.end(), x.src) == from.end()) {
        from.push_back(x.src);
        if (flags_) {
          hip_ok(hipStreamWaitValue32(s, flags_mine_ + x.src * kCh + ch, ++recv_seq_[x.src][ch],
                                      hipStreamWaitValueGte, 0xffffffffu),
                 "hipStreamWaitValue32");
        } else {
          int msg = -1;
          c_->recv(&msg, sizeof msg, x.src);
          if (msg != ch * 2 + par) throw std::runtime_error("peer transport: out-of-order note");
          hip_ok(hipStreamWaitEvent(s, peer_sent_[x.src][ch][par], 0), "hipStreamWaitEvent IPC");
        }
      }
      if (halo) {
        const int seq = x.seq >= 0 ? x.seq : static_cast<int>(i);
        copy2d(at(par, x.to), x.to.pitch, static_cast<char*>(slot_.at({seq, par})) + x.img0 * x.width, x.width,
               x.width, x.height, s);
      }
    }
  }

  // Collective: unmap every peer's buffers, wait for every rank to have done so, then free this
  // rank's own (a mapped peer buffer must not be freed under its importer).
  void close() override {
    const bool collective = connected_ && c_ && c_->size() > 1;
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    if (collective) c_->barrier();
    release();
  }
  void abort() override {
    // flags mode: raise this rank's words (its own waits return) and its words on every peer (their
    // waits on this rank return); a raised word satisfies every later >= wait too. Synchronous host
    // writes, not on a stream that may itself be parked in a wait.
    if (!flags_ || !flags_mine_) return;
    const std::vector<uint32_t> top(static_cast<size_t>(np_) * kCh, 0xffffffffu);
    (void)hipMemcpy(flags_mine_, top.data(), top.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    for (int r = 0; r < np_; ++r)
      if (r != rank_ && r < static_cast<int>(flags_of_.size()) && flags_of_[r])
        (void)hipMemcpy(flags_of_[r] + rank_ * kCh, top.data(), kCh * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  void release() {
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    for (hipEvent_t e : opened_ev_) (void)hipEventDestroy(e);
    opened_ev_.clear();
    for (auto& kv : slot_) (void)hipFree(kv.second);
    slot_.clear();
    peer_slot_.clear();
    for (auto& ch : sent_)
      for (auto& e : ch)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    if (flags_mine_) (void)hipFree(flags_mine_), flags_mine_ = nullptr;
    flags_of_.clear();
    connected_ = false;
  }
};

// ---------------------------------------------------------------------------------------- host
struct HostTransport : Transport {
  HostComm* hc_;
  int rank_;
  void* buf_[2][kB] = {};
  std::map<std::pair<int, int>, std::vector<char>> stage_;  // (phase, transfer index) -> packed bytes
  HostTransport(HostComm* c, int rank) : hc_(c), rank_(rank) {}
  const char* name() const override { return "host"; }
  const char* ordering() const override { return "blocking"; }
  char* at(int par, const Region& r) const { return static_cast<char*>(buf_[par][static_cast<int>(r.buf)]) + r.off; }
  static void copy2d(char* dst, size_t dpitch, const char* src, size_t spitch, size_t w, size_t h) {
    for (size_t i = 0; i < h; ++i) std::memcpy(dst + i * dpitch, src + i * spitch, w);
  }
  void bind(const Schedule&, void* const bufs[2][kB], hipStream_t) override {
    for (int p = 0; p < 2; ++p)
      for (int b = 0; b < kB; ++b) buf_[p][b] = bufs[p][b];
  }
  void bcast(void* buf, size_t bytes, int root) override {
    if (!record_only && hc_ && hc_->size() > 1) hc_->bcast(buf, bytes, root);
  }
  void run_phase(Phase ph, const std::vector<Transfer>& xs, hipStream_t, int par) override {
    std::vector<std::pair<const Transfer*, std::vector<char>*>> unpack;
    for (size_t i = 0; i < xs.size(); ++i) {
      const Transfer& x = xs[i];
      if (x.src != rank_ && x.dst != rank_) continue;
      note(x);
      if (record_only) continue;
      if (x.src == x.dst) {
        if (at(par, x.to) != at(par, x.from))
          copy2d(at(par, x.to), x.to.pitch, at(par, x.from), x.from.pitch, x.width, x.height);
        continue;
      }
      std::vector<char>& st = stage_[{static_cast<int>(ph), static_cast<int>(i)}];
      st.resize(x.bytes());
      if (x.src == rank_) {
        copy2d(st.data(), x.width, at(par, x.from), x.from.pitch, x.width, x.height);
        hc_->isend(st.data(), x.bytes(), x.dst);
      } else {
        hc_->irecv(st.data(), x.bytes(), x.src);
        unpack.push_back({&x, &st});
      }
    }
    if (record_only) return;
    hc_->wait_all();
    for (auto& u : unpack)
      copy2d(at(par, u.first->to), u.first->to.pitch, u.second->data(), u.first->width, u.first->width, u.first->height);
  }
};

}  // namespace

std::unique_ptr<Transport> make_host_transport(HostComm* c, int rank) { return std::make_unique<HostTransport>(c, rank); }

std::unique_ptr<Transport> make_rccl_transport(HostComm* c, int device, int rank, bool loopback) {
  return std::make_unique<RcclTransport>(c, device, rank, loopback);
}
std::unique_ptr<Transport> make_peer_transport(HostComm* c, int device, int rank, const std::string& sync) {
  return std::make_unique<PeerTransport>(c, device, rank, sync);
}

}  // namespace anx
