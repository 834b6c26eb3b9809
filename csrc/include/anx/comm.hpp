// anx/comm.hpp — the native communication layer of the anx CLI.
//
// Replaces the reference's Open MPI usage:
//   * HostComm  — host-memory message passing between ranks over TCP sockets (full mesh, bootstrap
//                 through rank 0). Used by the CPU versions (V2.1/V2.2), by V4's host staging, and
//                 to bootstrap RCCL. Point-to-point ops are queued in a group and progressed
//                 together with poll(), so a halo exchange in both directions cannot deadlock
//                 (the reference relies on MPI_Isend/Irecv + Waitall for the same).
//   * DeviceComm — RCCL communicator over xGMI for device buffers (V5): broadcast, grouped
//                 send/recv on a dedicated comm stream, ordered against the compute stream by
//                 events.
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

// RCCL communicator (V5). Built from a HostComm used only for the unique-id bootstrap.
class DeviceComm {
 public:
  DeviceComm(HostComm& boot, int device);
  ~DeviceComm();
  DeviceComm(const DeviceComm&) = delete;
  DeviceComm& operator=(const DeviceComm&) = delete;
  hipStream_t stream() const { return stream_; }
  void group_start();
  void group_end();
  void send(const void* buf, size_t bytes, int dst);
  void recv(void* buf, size_t bytes, int src);
  void bcast(void* buf, size_t bytes, int root);
  // Make `other` wait for everything queued on the comm stream so far (and vice versa).
  void after(hipStream_t compute);   // comm stream waits for compute
  void before(hipStream_t compute);  // compute waits for comm stream
  void abort();

 private:
  void* comm_ = nullptr;  // ncclComm_t
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_ = nullptr;
};

}  // namespace anx
