// anx_dgemm — the reference's homework-1 workload: C = A.B for n x n fp64
// matrices with the rows of A distributed over ranks, B broadcast, C gathered on rank 0 and checked
// against a serial recomputation (tolerance 1e-6). Reference: homeworks/hw1/src/template.c:30-238
// (MPI_Send/Recv scatter :121-129, MPI_Bcast B :132, gather :138-146, check :157-175).
//
//   anxrun -np P anx_dgemm <n> [--gpu] [--seed S]
//
// n must be a power of two, <= 4096 (larger is clamped, as the reference does) and divisible by P.
// With --gpu each rank multiplies its row block on its GPU (LOCAL_RANK % #devices) with an fp64
// MFMA kernel (v_mfma_f64_16x16x4_f64); otherwise a cache-blocked host loop.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "anx/comm.hpp"

namespace {

constexpr int kMaxDim = 4096;

// One wave per 16x16 C tile, 4 waves (2x2) per workgroup = a 32x32 tile.
// f64 MFMA fragment maps (cdna guide §3): A[i=l&15][k=l>>4], B[k=l>>4][j=l&15];
// D: col = l&15, row = (l>>4) + 4*reg.
__global__ void __launch_bounds__(256) dgemm_mfma(const double* __restrict__ A, const double* __restrict__ B,
                                                  double* __restrict__ C, int rows, int n) {
  using f64x4 = __attribute__((ext_vector_type(4))) double;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i0 = blockIdx.y * 32 + (wave >> 1) * 16, j0 = blockIdx.x * 32 + (wave & 1) * 16;
  const int li = lane & 15, lk = lane >> 4;
  f64x4 acc = {0, 0, 0, 0};
  const int ai = i0 + li < rows ? i0 + li : rows - 1;
  for (int k = 0; k < n; k += 4) {
    const double a = A[static_cast<size_t>(ai) * n + k + lk];
    const double b = B[static_cast<size_t>(k + lk) * n + j0 + li];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + lk + 4 * r;
    if (i < rows) C[static_cast<size_t>(i) * n + j0 + li] = acc[r];
  }
}

void hip_check(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string(w) + ": " + hipGetErrorString(e));
}

void host_mm(const double* a, const double* b, double* c, int rows, int n) {
  std::memset(c, 0, sizeof(double) * rows * n);
  constexpr int T = 64;
  for (int i0 = 0; i0 < rows; i0 += T)
    for (int k0 = 0; k0 < n; k0 += T)
      for (int i = i0; i < std::min(rows, i0 + T); ++i)
        for (int k = k0; k < std::min(n, k0 + T); ++k) {
          const double av = a[static_cast<size_t>(i) * n + k];
          const double* br = b + static_cast<size_t>(k) * n;
          double* cr = c + static_cast<size_t>(i) * n;
          for (int j = 0; j < n; ++j) cr[j] += av * br[j];
        }
}

}  // namespace

int main(int argc, char** argv) {
  int n = 1024;
  bool gpu = false;
  unsigned seed = 1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--gpu") gpu = true;
    else if (a == "--seed" && i + 1 < argc) seed = static_cast<unsigned>(std::atoi(argv[++i]));
    else n = std::atoi(argv[i]);
  }
  const anx::RankInfo ri = anx::rank_info_from_env();
  anx::HostComm c(ri);
  const int rank = c.rank(), np = c.size();
  if (n <= 0 || (n & (n - 1)) != 0) {
    if (rank == 0) std::fprintf(stderr, "Error: matrix dimension n (%d) must be a positive power of two\n", n);
    c.abort("bad n");
  }
  if (n > kMaxDim) {
    if (rank == 0) std::fprintf(stderr, "Warning: n (%d) exceeds %d, clamping\n", n, kMaxDim);
    n = kMaxDim;
  }
  if (n % np != 0) {
    if (rank == 0) std::fprintf(stderr, "Error: n (%d) must be divisible by the number of ranks (%d)\n", n, np);
    c.abort("bad n/np");
  }
  const int rows = n / np;
  const size_t nn = static_cast<size_t>(n) * n, rn = static_cast<size_t>(rows) * n;
  std::vector<double> A, B(nn), C, a(rn), cl(rn);
  if (rank == 0) {
    A.resize(nn);
    C.resize(nn);
    std::srand(seed);
    for (size_t i = 0; i < nn; ++i) A[i] = static_cast<double>(std::rand() % 10);
    for (size_t i = 0; i < nn; ++i) B[i] = static_cast<double>(std::rand() % 10);
  }
  c.barrier();
  const auto t0 = std::chrono::steady_clock::now();
  // scatter row blocks of A, broadcast B
  if (rank == 0) {
    std::memcpy(a.data(), A.data(), rn * sizeof(double));
    for (int r = 1; r < np; ++r) c.isend(A.data() + r * rn, rn * sizeof(double), r);
    c.wait_all();
  } else {
    c.recv(a.data(), rn * sizeof(double), 0);
  }
  c.bcast(B.data(), nn * sizeof(double), 0);
  if (gpu) {
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev < 1) c.abort("--gpu needs a GPU");
    hip_check(hipSetDevice(ri.local_rank % ndev), "hipSetDevice");
    double *dA, *dB, *dC;
    hip_check(hipMalloc(&dA, rn * 8), "malloc");
    hip_check(hipMalloc(&dB, nn * 8), "malloc");
    hip_check(hipMalloc(&dC, rn * 8), "malloc");
    hip_check(hipMemcpy(dA, a.data(), rn * 8, hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(dB, B.data(), nn * 8, hipMemcpyHostToDevice), "H2D");
    dgemm_mfma<<<dim3(n / 32, (rows + 31) / 32), 256>>>(dA, dB, dC, rows, n);
    hip_check(hipGetLastError(), "launch");
    hip_check(hipMemcpy(cl.data(), dC, rn * 8, hipMemcpyDeviceToHost), "D2H");
    (void)hipFree(dA);
    (void)hipFree(dB);
    (void)hipFree(dC);
  } else {
    host_mm(a.data(), B.data(), cl.data(), rows, n);
  }
  // gather C row blocks on rank 0
  if (rank == 0) {
    std::memcpy(C.data(), cl.data(), rn * sizeof(double));
    for (int r = 1; r < np; ++r) c.irecv(C.data() + r * rn, rn * sizeof(double), r);
    c.wait_all();
  } else {
    c.send(cl.data(), rn * sizeof(double), 0);
  }
  c.barrier();
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int bad = 0;
  if (rank == 0) {
    std::vector<double> D(nn);
    host_mm(A.data(), B.data(), D.data(), n, n);
    for (size_t i = 0; i < nn && !bad; ++i)
      if (std::fabs(C[i] - D[i]) > 1e-6) {
        std::printf("ERROR: Mismatch at C[%zu][%zu]=%f != %f\n", i / n, i % n, C[i], D[i]);
        bad = 1;
      }
    std::printf("n=%d np=%d %s time %.6f s, %.2f GFLOP/s: %s\n", n, np, gpu ? "gpu" : "cpu", secs,
                2.0 * n * static_cast<double>(n) * n / secs / 1e9, bad ? "FAILED" : "Result verified");
    std::printf("ANX_JSON {\"version\": \"hw1_dgemm\", \"np\": %d, \"n\": %d, \"gpu\": %s, \"time_s\": %.6f, "
                "\"ok\": %s}\n",
                np, n, gpu ? "true" : "false", secs, bad ? "false" : "true");
  }
  c.barrier();
  return bad;
}
