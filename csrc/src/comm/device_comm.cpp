// DeviceComm: RCCL over xGMI for device-resident V5 traffic (see anx/comm.hpp).
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>

#include "anx/comm.hpp"

namespace anx {

namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP ") + what + ": " + hipGetErrorString(e));
}
ncclComm_t C(void* p) { return static_cast<ncclComm_t>(p); }
}  // namespace

DeviceComm::DeviceComm(HostComm& boot, int device) {
  hip_check(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId id;
  if (boot.rank() == 0) nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  boot.bcast(&id, sizeof id, 0);
  ncclComm_t c;
  nccl_check(ncclCommInitRank(&c, boot.size(), id, boot.rank()), "ncclCommInitRank");
  comm_ = c;
  hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
  hip_check(hipEventCreateWithFlags(&ev_, hipEventDisableTiming), "hipEventCreate");
}

DeviceComm::~DeviceComm() {
  if (comm_) ncclCommDestroy(C(comm_));
  if (ev_) (void)hipEventDestroy(ev_);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void DeviceComm::group_start() { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
void DeviceComm::group_end() { nccl_check(ncclGroupEnd(), "ncclGroupEnd"); }

void DeviceComm::send(const void* buf, size_t bytes, int dst) {
  if (bytes) nccl_check(ncclSend(buf, bytes, ncclChar, dst, C(comm_), stream_), "ncclSend");
}
void DeviceComm::recv(void* buf, size_t bytes, int src) {
  if (bytes) nccl_check(ncclRecv(buf, bytes, ncclChar, src, C(comm_), stream_), "ncclRecv");
}
void DeviceComm::bcast(void* buf, size_t bytes, int root) {
  nccl_check(ncclBroadcast(buf, buf, bytes, ncclChar, root, C(comm_), stream_), "ncclBroadcast");
}

void DeviceComm::after(hipStream_t compute) {
  hip_check(hipEventRecord(ev_, compute), "hipEventRecord");
  hip_check(hipStreamWaitEvent(stream_, ev_, 0), "hipStreamWaitEvent");
}
void DeviceComm::before(hipStream_t compute) {
  hip_check(hipEventRecord(ev_, stream_), "hipEventRecord");
  hip_check(hipStreamWaitEvent(compute, ev_, 0), "hipStreamWaitEvent");
}

void DeviceComm::abort() {
  if (comm_) ncclCommAbort(C(comm_));
  comm_ = nullptr;
}

}  // namespace anx
