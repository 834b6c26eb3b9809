// anx/comm.hpp — the native communication layer of the anx CLI.
//
// Replaces the reference's Open MPI usage:
//   * HostComm  — host-memory message passing between ranks over TCP sockets (full mesh, bootstrap
//                 through rank 0). Used by the CPU versions (V2.1/V2.2), by V4's host staging, and
//                 to bootstrap RCCL. Point-to-point ops are queued in a group and progressed
//                 together with poll(), so a halo exchange in both directions cannot deadlock
//                 (the reference relies on MPI_Isend/Irecv + Waitall for the same).
//   * DeviceComm — device-buffer communicator (V5): RCCL over xGMI, or a loopback implementation of
//                 the same contract for ranks sharing one GPU; broadcast, grouped send/recv on a
//                 dedicated comm stream, ordered against the compute stream by events.
// Rank/world come from ANX_RANK/ANX_WORLD_SIZE (set by anxrun) or RANK/WORLD_SIZE (torchrun);
// rendezvous at ANX_MASTER_ADDR:ANX_MASTER_PORT (or MASTER_ADDR/MASTER_PORT), default 127.0.0.1.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace anx {

struct RankInfo {
  int rank = 0, world = 1, local_rank = 0;
  int local_world = 1;  // ranks on this node (ANX_LOCAL_WORLD_SIZE / LOCAL_WORLD_SIZE; default: world)
  int nnodes = 1;       // nodes in the job (ANX_NNODES / world / local_world)
  std::string master_addr = "127.0.0.1";
  int master_port = 29555;
};
RankInfo rank_info_from_env();

class HostComm {
 public:
  explicit HostComm(const RankInfo& ri, double timeout_s = 300.0);
  ~HostComm();
  HostComm(const HostComm&) = delete;
  HostComm& operator=(const HostComm&) = delete;

  int rank() const { return rank_; }
  int size() const { return world_; }

  // Point-to-point, grouped: queue with isend/irecv, run them all with wait_all().
  void isend(const void* buf, size_t bytes, int dst);
  void irecv(void* buf, size_t bytes, int src);
  void wait_all();
  void send(const void* buf, size_t bytes, int dst) { isend(buf, bytes, dst), wait_all(); }
  void recv(void* buf, size_t bytes, int src) { irecv(buf, bytes, src), wait_all(); }

  // Collectives built on P2P (root-centred; world sizes here are single-node, <= a few dozen).
  void barrier();
  void bcast(void* buf, size_t bytes, int root);
  void allreduce_max(double* v, int n);
  // Abort every rank: close sockets; peers blocked in wait_all() fail fast ("MPI_Abort").
  [[noreturn]] void abort(const std::string& why, int code = 1);

 private:
  struct Op {
    int peer;
    char* p;
    size_t left;
    bool send;
  };
  int rank_, world_;
  double timeout_s_;
  std::vector<int> fd_;  // socket per peer (-1 for self)
  std::vector<Op> ops_;
};

// Device communicator (V5): grouped send/recv and broadcast of device buffers on a dedicated comm
// stream, ordered against compute streams by events. Two implementations behind one interface:
//   rccl      — an RCCL communicator over xGMI (one GPU per rank);
//   loopback  — the same contract for ranks that SHARE a GPU (RCCL refuses two ranks on one device):
//               group_end matches the queued sends / receives through the host channel (the receiver
//               sends the IPC handle + offset of each receive buffer), the sender's comm stream waits
//               for the receiver's "posted" flag, copies straight into the receiver's IPC-mapped
//               buffer (hipMemcpyAsync) and raises a "landed" flag the receiver's comm stream waits
//               for (hipStreamWriteValue32 / hipStreamWaitValue32 on IPC-shared words). It exists so
//               the RCCL transport's pack / staging / grouped P2P / unpack / two-communicator code
//               runs unchanged, multi-rank, on a one-GPU box.
class DeviceComm {
 public:
  virtual ~DeviceComm() = default;
  virtual const char* kind() const = 0;  // "rccl" | "loopback"
  virtual hipStream_t stream() const = 0;
  virtual void group_start() = 0;
  virtual void group_end() = 0;
  virtual void send(const void* buf, size_t bytes, int dst) = 0;
  virtual void recv(void* buf, size_t bytes, int src) = 0;
  virtual void bcast(void* buf, size_t bytes, int root) = 0;
  // Make the comm stream wait for everything queued on `compute` so far / the reverse.
  void after(hipStream_t compute);   // comm stream waits for compute
  void before(hipStream_t compute);  // compute waits for comm stream
  // Make this comm stream wait for everything queued on `other`'s comm stream so far: two
  // communicators of one rank then run in one total order, the same on every rank (their ops are
  // issued in the same host order everywhere), so neither can wait on a peer that is itself stuck
  // behind the other communicator.
  void after_comm(DeviceComm& other);
  virtual void abort() {}

 protected:
  void init_sync();  // creates ev_ (call from the implementations' constructors)
  hipEvent_t ev_ = nullptr;
};
// Collective over `boot` (every rank constructs its communicators in the same order).
std::unique_ptr<DeviceComm> make_rccl_comm(HostComm& boot, int device);
std::unique_ptr<DeviceComm> make_loopback_comm(HostComm& boot, int device);

}  // namespace anx
