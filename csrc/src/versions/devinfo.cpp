// anx_devinfo — per-rank device binding report (the reference's MPI+CUDA homework template,
// rank -> GPU `rank % num_devices`, cudaSetDevice, device-properties print,
// templates/template.cu.template:43-51). Run under `anxrun -np N anx_devinfo`.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "anx/comm.hpp"

int main() {
  const anx::RankInfo ri = anx::rank_info_from_env();
  anx::HostComm c(ri);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  char line[512];
  if (ndev > 0) {
    const int dev = ri.local_rank % ndev;
    (void)hipSetDevice(dev);
    hipDeviceProp_t p{};
    (void)hipGetDeviceProperties(&p, dev);
    std::snprintf(line, sizeof line,
                  "rank %d/%d local %d -> device %d/%d: %s (%s) CUs %d, %.1f GB HBM, LDS/block %zu KB, wave %d, "
                  "clock %.2f GHz, PCI %02x:%02x",
                  c.rank(), c.size(), ri.local_rank, dev, ndev, p.name, p.gcnArchName, p.multiProcessorCount,
                  p.totalGlobalMem / 1e9, p.sharedMemPerBlock / 1024, p.warpSize, p.clockRate / 1e6, p.pciBusID,
                  p.pciDeviceID);
  } else {
    std::snprintf(line, sizeof line, "rank %d/%d local %d -> no GPU visible", c.rank(), c.size(), ri.local_rank);
  }
  // ordered print through rank 0
  char buf[512];
  if (c.rank() == 0) {
    std::puts(line);
    for (int r = 1; r < c.size(); ++r) {
      c.recv(buf, sizeof buf, r);
      std::puts(buf);
    }
  } else {
    c.send(line, sizeof line, 0);
  }
  c.barrier();
  return 0;
}
