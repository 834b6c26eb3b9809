// Device communicators for device-resident V5 traffic (see anx/comm.hpp): RCCL over xGMI, and the
// loopback implementation of the same contract for ranks that share one GPU.
//
// Reference call sites these replace: the V4 scatter / halo / gather MPI calls
// (final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:61-62, 70-76, 129-130) and the planned V5's
// device pointers passed to MPI (README.md:158-166).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "anx/comm.hpp"

namespace anx {

namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

void DeviceComm::init_sync() { hip_check(hipEventCreateWithFlags(&ev_, hipEventDisableTiming), "hipEventCreate"); }

void DeviceComm::after(hipStream_t compute) {
  hip_check(hipEventRecord(ev_, compute), "hipEventRecord");
  hip_check(hipStreamWaitEvent(stream(), ev_, 0), "hipStreamWaitEvent");
}
void DeviceComm::before(hipStream_t compute) {
  hip_check(hipEventRecord(ev_, stream()), "hipEventRecord");
  hip_check(hipStreamWaitEvent(compute, ev_, 0), "hipStreamWaitEvent");
}
void DeviceComm::after_comm(DeviceComm& other) {
  if (&other == this) return;
  hip_check(hipEventRecord(other.ev_, other.stream()), "hipEventRecord");
  hip_check(hipStreamWaitEvent(stream(), other.ev_, 0), "hipStreamWaitEvent");
}

// ---------------------------------------------------------------------------------------------- RCCL
namespace {

class RcclComm final : public DeviceComm {
 public:
  RcclComm(HostComm& boot, int device) {
    hip_check(hipSetDevice(device), "hipSetDevice");
    ncclUniqueId id;
    if (boot.rank() == 0) nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    boot.bcast(&id, sizeof id, 0);
    ncclComm_t c;
    nccl_check(ncclCommInitRank(&c, boot.size(), id, boot.rank()), "ncclCommInitRank");
    comm_ = c;
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    init_sync();
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
    if (ev_) (void)hipEventDestroy(ev_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  const char* kind() const override { return "rccl"; }
  hipStream_t stream() const override { return stream_; }
  void group_start() override { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
  void group_end() override { nccl_check(ncclGroupEnd(), "ncclGroupEnd"); }
  void send(const void* buf, size_t bytes, int dst) override {
    if (bytes) nccl_check(ncclSend(buf, bytes, ncclChar, dst, comm_, stream_), "ncclSend");
  }
  void recv(void* buf, size_t bytes, int src) override {
    if (bytes) nccl_check(ncclRecv(buf, bytes, ncclChar, src, comm_, stream_), "ncclRecv");
  }
  void bcast(void* buf, size_t bytes, int root) override {
    nccl_check(ncclBroadcast(buf, buf, bytes, ncclChar, root, comm_, stream_), "ncclBroadcast");
  }
  void abort() override {
    if (comm_) ncclCommAbort(comm_);
    comm_ = nullptr;
  }

 private:
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
};

// ------------------------------------------------------------------------------------------ loopback
// Per peer pair, the i-th send of A to B matches the i-th receive of B from A (RCCL's P2P order).
// Flag words (device memory, IPC-shared, written by peers with hipStreamWriteValue32):
//   flags[src][0] on the SENDER  = how many receives from it the receiver's comm stream has posted
//   flags[src][1] on the RECEIVER = how many sends to it the sender's comm stream has landed
class LoopbackComm final : public DeviceComm {
 public:
  LoopbackComm(HostComm& boot, int device) : hc_(boot), rank_(boot.rank()), np_(boot.size()) {
    hip_check(hipSetDevice(device), "hipSetDevice");
    int can = 0;
    if (hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, device) != hipSuccess || !can)
      throw std::runtime_error("loopback device comm: the device lacks hipStreamWaitValue32");
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    init_sync();
    const size_t bytes = static_cast<size_t>(np_) * 2 * sizeof(uint32_t);
    hip_check(hipMalloc(reinterpret_cast<void**>(&flags_), bytes), "hipMalloc flags");
    hip_check(hipMemset(flags_, 0, bytes), "hipMemset flags");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    flags_of_.assign(np_, nullptr);
    for (int r = 0; r < np_; ++r) {  // collective: every rank's flag words mapped here
      hipIpcMemHandle_t h{};
      if (r == rank_) hip_check(hipIpcGetMemHandle(&h, flags_), "hipIpcGetMemHandle");
      hc_.bcast(&h, sizeof h, r);
      if (r == rank_) {
        flags_of_[r] = flags_;
      } else {
        void* p = nullptr;
        hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle flags");
        flags_of_[r] = static_cast<uint32_t*>(p);
        opened_.push_back(p);
      }
    }
    sent_.assign(np_, 0);
    posted_.assign(np_, 0);
  }
  ~LoopbackComm() override {
    try {
      (void)hipStreamSynchronize(stream_);
      if (!aborted_) hc_.barrier();  // no peer copies into our buffers or writes our flags any more
    } catch (...) {
    }
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    for (auto& kv : peer_bufs_) (void)hipIpcCloseMemHandle(kv.second);
    if (flags_) (void)hipFree(flags_);
    if (ev_) (void)hipEventDestroy(ev_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  const char* kind() const override { return "loopback"; }
  // RCCL's ncclCommAbort equivalent: a stream parked in hipStreamWaitValue32 on a peer that died would
  // never drain (and the destructor's stream sync would hang). Raise every flag word this rank waits
  // on, and its words on every peer, to the maximum (a >= wait then returns) with synchronous host
  // writes; skip the teardown barrier.
  void abort() override {
    aborted_ = true;
    if (!flags_) return;
    const std::vector<uint32_t> top(static_cast<size_t>(np_) * 2, 0xffffffffu);
    (void)hipMemcpy(flags_, top.data(), top.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    for (int r = 0; r < np_; ++r)
      if (r != rank_ && flags_of_[r]) (void)hipMemcpy(flags_of_[r] + rank_ * 2, top.data(), 2 * sizeof(uint32_t),
                                                       hipMemcpyHostToDevice);
  }
  hipStream_t stream() const override { return stream_; }
  void group_start() override {
    if (in_group_) throw std::runtime_error("loopback device comm: nested group");
    in_group_ = true;
  }
  void send(const void* buf, size_t bytes, int dst) override {
    if (bytes) ops_.push_back({true, const_cast<void*>(buf), bytes, dst});
    if (!in_group_) group_end();
  }
  void recv(void* buf, size_t bytes, int src) override {
    if (bytes) ops_.push_back({false, buf, bytes, src});
    if (!in_group_) group_end();
  }
  void bcast(void* buf, size_t bytes, int root) override {
    group_start();
    if (rank_ == root) {
      for (int r = 0; r < np_; ++r)
        if (r != root) send(buf, bytes, r);
    } else {
      recv(buf, bytes, root);
    }
    group_end();
  }
  void group_end() override {
    in_group_ = false;
    std::vector<Op> ops;
    ops.swap(ops_);
    if (ops.empty()) return;
    // 1. every receive: post it on the comm stream (the sender may write once our stream got here) and
    // tell the sender where its bytes go
    std::vector<Meta> out, in;
    out.reserve(ops.size());
    in.reserve(ops.size());
    for (const Op& o : ops) {
      if (o.send) continue;
      Meta m{};
      void* base = nullptr;
      size_t size = 0;
      hip_check(hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t*>(&base), &size, o.buf), "hipMemGetAddressRange");
      auto hit = my_handles_.find(base);  // one handle per allocation (every buffer here outlives the comm)
      if (hit == my_handles_.end()) {
        hipIpcMemHandle_t h{};
        hip_check(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
        hit = my_handles_.emplace(base, h).first;
      }
      m.handle = hit->second;
      m.offset = static_cast<uint64_t>(static_cast<char*>(o.buf) - static_cast<char*>(base));
      m.bytes = o.bytes;
      m.seq = ++posted_[o.peer];
      out.push_back(m);
      hip_check(hipStreamWriteValue32(stream_, flags_of_[o.peer] + rank_ * 2 + 0, m.seq, 0), "hipStreamWriteValue32");
    }
    size_t oi = 0;
    for (const Op& o : ops) {
      if (o.send) continue;
      hc_.isend(&out[oi++], sizeof(Meta), o.peer);
    }
    for (const Op& o : ops)
      if (o.send) {
        in.push_back(Meta{});
        hc_.irecv(&in.back(), sizeof(Meta), o.peer);
      }
    hc_.wait_all();
    // 2. every send: wait until the receiver posted it, copy into its buffer, raise its landed flag
    size_t ii = 0;
    for (const Op& o : ops) {
      if (!o.send) continue;
      const Meta& m = in[ii++];
      const uint32_t seq = ++sent_[o.peer];
      if (m.seq != seq || m.bytes != o.bytes)
        throw std::runtime_error("loopback device comm: send #" + std::to_string(seq) + " to rank " +
                                 std::to_string(o.peer) + " (" + std::to_string(o.bytes) + " B) met receive #" +
                                 std::to_string(m.seq) + " (" + std::to_string(m.bytes) + " B)");
      char* dst = static_cast<char*>(open(o.peer, m.handle)) + m.offset;
      hip_check(hipStreamWaitValue32(stream_, flags_ + o.peer * 2 + 0, seq, hipStreamWaitValueGte, 0xffffffffu),
                "hipStreamWaitValue32");
      hip_check(hipMemcpyAsync(dst, o.buf, o.bytes, hipMemcpyDeviceToDevice, stream_), "hipMemcpyAsync");
      hip_check(hipStreamWriteValue32(stream_, flags_of_[o.peer] + rank_ * 2 + 1, seq, 0), "hipStreamWriteValue32");
    }
    // 3. every receive completes when its sender's copy landed
    for (const Op& o : ops)
      if (!o.send) {
        landed_wait_[o.peer] += 1;
        hip_check(hipStreamWaitValue32(stream_, flags_ + o.peer * 2 + 1, landed_wait_[o.peer], hipStreamWaitValueGte,
                                       0xffffffffu),
                  "hipStreamWaitValue32");
      }
  }

 private:
  struct Op {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
  };
  struct Meta {
    hipIpcMemHandle_t handle;
    uint64_t offset, bytes;
    uint32_t seq, pad;
  };
  void* open(int peer, const hipIpcMemHandle_t& h) {
    std::string key(reinterpret_cast<const char*>(&h), sizeof h);
    key += std::to_string(peer);
    auto it = peer_bufs_.find(key);
    if (it != peer_bufs_.end()) return it->second;
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    peer_bufs_[key] = p;
    return p;
  }

  HostComm& hc_;
  int rank_, np_;
  hipStream_t stream_ = nullptr;
  uint32_t* flags_ = nullptr;
  std::vector<uint32_t*> flags_of_;
  std::vector<void*> opened_;
  std::map<std::string, void*> peer_bufs_;
  std::map<void*, hipIpcMemHandle_t> my_handles_;
  std::vector<uint32_t> sent_, posted_;
  std::map<int, uint32_t> landed_wait_;
  std::vector<Op> ops_;
  bool in_group_ = false;
  bool aborted_ = false;
};

}  // namespace

std::unique_ptr<DeviceComm> make_rccl_comm(HostComm& boot, int device) { return std::make_unique<RcclComm>(boot, device); }
std::unique_ptr<DeviceComm> make_loopback_comm(HostComm& boot, int device) {
  return std::make_unique<LoopbackComm>(boot, device);
}

}  // namespace anx
