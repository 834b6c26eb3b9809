// anx — the native CLI: the reference's five staged programs in one binary.
//
//   anx --version v1|v2.1|v2.2|v3|v4|v5 [--batch N] [--init const|rand] [--seed S]
//       [--lrn-alpha-mode div_n|raw] [--groups 1|2] [--decomp overlap|per_layer] [--iters K]
//       [--impl mfma|direct] [--check] [--no-json]
//
// Multi-rank versions run under `anxrun -np N anx ...` (or torchrun-style RANK/WORLD_SIZE env).
// Each run prints the reference's stdout contract and one `ANX_JSON {...}` line with
// cold (first call incl. setup, like the reference's timers) and warm (steady-state mean) timings,
// per-phase breakdown, checksum (CRC-32 of the fp32 output, identical to the Python package's) and,
// with --check, the max error vs a single-process host recomputation.
//
// Reference programs: v1_serial/src/main.cpp:10-78, v2_mpi_only/2.1_broadcast_all/src/main.cpp:10-109,
// v2_mpi_only/2.2_scatter_halo/src/main.cpp:23-290, v3_cuda_only/src/main_cuda.cpp:12-44,
// v4_mpi_cuda/src/main_mpi_cuda.cpp:20-163; V5 is empty in the reference (README.md:158-166).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "anx/comm.hpp"
#include "anx/cpu_engine.hpp"
#include "anx/engine.hpp"
#include "anx/upload.hpp"
#include "anx/plan.hpp"
#include "anx/rng.hpp"
#include "anx/schedule.hpp"
#include "anx/trace.hpp"
#include "anx/v5.hpp"

using namespace anx;

namespace {

struct Options {
  std::string version = "v3";
  int batch = 1;
  std::string init = "const";
  unsigned seed = 0;
  std::string lrn;     // "" = version default
  int groups = 1;
  std::string decomp;  // "" = version default
  int iters = 0;
  std::string impl = "mfma";
  std::string conv2_algo = "auto";  // auto | direct | winograd
  std::string conv1_algo = "auto";  // auto | direct | winograd
  std::string transport = "auto";   // v5 device traffic: auto | rccl | peer (IPC + hipMemcpy2DAsync) | loopback
  std::string split = "auto";       // v5 decomposition: auto (cost model) | rows (reference) | hybrid | batch
  std::string input_source = "local";  // v5: local (device-resident, placed once) | root (scattered every step)
  int lanes = 0;                    // v5: stream lanes of a halo-free rank (0 = the runtime's default)
  int chunks = 0;                   // v5: halo pipeline chunks per step (0 = auto)
  int row_ways = 0;                 // v5: explicit row split (ranks per row group; 0 = from --split)
  std::string peer_sync;            // v5 peer transport ordering: flags | notes ("" = default)
  bool dry_run = false;             // v5: print the transfer schedule (record-only transports, no GPU)
  std::string pipeline = "auto";    // v5: scatter / gather on a second stream (auto: on over RCCL)
  bool poison = false;              // v5: NaN-fill consumed buffers (a mis-ordered step corrupts the output)
  bool check = false;
  bool json = true;
  std::string weights;  // directory with raw fp32 w1/b1/w2/b2 .bin (overrides --init for weights)
};

[[noreturn]] void usage(const char* msg) {
  std::fprintf(stderr,
               "%s\nusage: anx --version v1|v2.1|v2.2|v3|v4|v5 [--batch N] [--init const|rand] [--seed S]\n"
               "           [--lrn-alpha-mode div_n|raw] [--groups 1|2] [--decomp overlap|per_layer]\n"
               "           [--iters K] [--impl mfma|direct] [--conv2-algo auto|direct|winograd]\n"
               "           [--conv1-algo auto|direct|winograd] [--transport auto|rccl|peer|loopback] [--check]\n"
               "           [--split auto|rows|hybrid|batch] [--row-ways R] [--chunks K] [--peer-sync flags|notes]\n"
               "           [--input-source local|root] [--lanes L]\n"
               "           [--dry-run] [--pipeline auto|on|off] [--poison]\n"
               "           [--weights DIR] [--no-json]\n",
               msg);
  std::exit(2);
}

Options parse(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) usage(("missing value for " + a).c_str());
      return argv[++i];
    };
    if (a == "--version" || a == "-v") o.version = val();
    else if (a == "--batch" || a == "-b") o.batch = std::atoi(val().c_str());
    else if (a == "--init") o.init = val();
    else if (a == "--seed") o.seed = static_cast<unsigned>(std::atoi(val().c_str()));
    else if (a == "--lrn-alpha-mode") o.lrn = val();
    else if (a == "--groups") o.groups = std::atoi(val().c_str());
    else if (a == "--decomp") o.decomp = val();
    else if (a == "--iters") o.iters = std::atoi(val().c_str());
    else if (a == "--impl") o.impl = val();
    else if (a == "--conv2-algo") o.conv2_algo = val();
    else if (a == "--conv1-algo") o.conv1_algo = val();
    else if (a == "--transport") o.transport = val();
    else if (a == "--split") o.split = val();
    else if (a == "--row-ways") o.row_ways = std::atoi(val().c_str());
    else if (a == "--input-source") o.input_source = val();
    else if (a == "--lanes") o.lanes = std::atoi(val().c_str());
    else if (a == "--chunks") o.chunks = std::atoi(val().c_str());
    else if (a == "--peer-sync") o.peer_sync = val();
    else if (a == "--dry-run") o.dry_run = true;
    else if (a == "--pipeline") {
      o.pipeline = val();
      if (o.pipeline != "on" && o.pipeline != "off" && o.pipeline != "auto") usage("--pipeline must be auto, on or off");
    } else if (a == "--poison") o.poison = true;
    else if (a == "--check") o.check = true;
    else if (a == "--no-json") o.json = false;
    else if (a == "--weights") o.weights = val();
    else if (a == "-h" || a == "--help") usage("");
    else usage(("unknown argument " + a).c_str());
  }
  static const char* vs[] = {"v1", "v2.1", "v2.2", "v3", "v4", "v5"};
  if (std::find(std::begin(vs), std::end(vs), o.version) == std::end(vs)) usage("bad --version");
  if (o.lrn.empty()) o.lrn = (o.version == "v1" || o.version == "v2.1" || o.version == "v2.2") ? "div_n" : "raw";
  if (o.decomp.empty()) o.decomp = o.version == "v5" ? "per_layer" : "overlap";
  if (o.batch < 1) usage("--batch must be >= 1");
  if (o.split != "auto" && o.split != "rows" && o.split != "hybrid" && o.split != "batch") usage("bad --split");
  if (o.chunks < 0) usage("--chunks must be >= 0");
  if (o.row_ways < 0) usage("--row-ways must be >= 0");
  if (o.input_source != "local" && o.input_source != "root") usage("--input-source must be local or root");
  if (o.lanes < 0) usage("--lanes must be >= 0");
  if (!o.peer_sync.empty() && o.peer_sync != "flags" && o.peer_sync != "notes") usage("--peer-sync must be flags or notes");
  return o;
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

uint32_t crc32(const void* data, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  uint32_t c = 0xFFFFFFFFu;
  const auto* p = static_cast<const unsigned char*>(data);
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Ordered phase accumulator.
struct Phases {
  std::vector<std::pair<std::string, double>> v;
  void add(const std::string& k, double ms) {
    for (auto& p : v)
      if (p.first == k) {
        p.second += ms;
        return;
      }
    v.push_back({k, ms});
  }
  double total() const {
    double t = 0;
    for (auto& p : v) t += p.second;
    return t;
  }
  std::string json(double scale = 1.0) const {
    std::string s = "{";
    char buf[96];
    for (size_t i = 0; i < v.size(); ++i) {
      std::snprintf(buf, sizeof buf, "%s\"%s\": %.4f", i ? ", " : "", v[i].first.c_str(), v[i].second * scale);
      s += buf;
    }
    return s + "}";
  }
};

// Copy `nrows` rows (each `row_floats`) of N images between row-windowed buffers: image n of src holds
// rows [0, src_rows) with the copied block starting at src_off; dst likewise. Host or device.
void copy_rows(float* dst, int dst_rows, int dst_off, const float* src, int src_rows, int src_off, int nrows,
               size_t row_floats, int N, bool device, hipStream_t s) {
  if (nrows <= 0 || N <= 0) return;
  const size_t w = static_cast<size_t>(nrows) * row_floats * sizeof(float);
  const size_t dp = static_cast<size_t>(dst_rows) * row_floats * sizeof(float);
  const size_t sp = static_cast<size_t>(src_rows) * row_floats * sizeof(float);
  float* d = dst + static_cast<size_t>(dst_off) * row_floats;
  const float* q = src + static_cast<size_t>(src_off) * row_floats;
  if (device) {
    hip_check(hipMemcpy2DAsync(d, dp, q, sp, w, N, hipMemcpyDeviceToDevice, s), "hipMemcpy2DAsync");
  } else {
    for (int n = 0; n < N; ++n)
      std::memcpy(reinterpret_cast<char*>(d) + n * dp, reinterpret_cast<const char*>(q) + n * sp, w);
  }
}

struct Setup {
  Options o;
  Knobs k;  // engine kernel knobs (--conv1-algo / --conv2-algo over default_knobs())
  RankInfo ri;
  BlockSpec b1, b2;
  BlocksDims d;
  HostWeights w;
  std::vector<float> x;  // full input (rank 0; every rank for v2.1)
  size_t in_row, out_row;
};

Setup make_setup(const Options& o, const RankInfo& ri) {
  Setup s;
  s.o = o;
  s.ri = ri;
  s.k = default_knobs();
  // Winograd conv2 sums in a different order per row tile (tile origins move with the decomposition):
  // results match to ~1e-7 relative, not bitwise; `direct` makes every decomposition bit-identical.
  // Conv1 likewise: polyphase Winograd by default, `direct` for bit-identical decompositions.
  auto algo = [](const std::string& a, ConvAlgo dflt) {
    return a == "direct" ? ConvAlgo::Direct : a == "winograd" ? ConvAlgo::Winograd : dflt;
  };
  s.k.conv2_algo = algo(o.conv2_algo, s.k.conv2_algo);
  s.k.conv1_algo = algo(o.conv1_algo, s.k.conv1_algo);
  s.b1 = kBlock1;
  s.b2 = kBlock2;
  s.b2.conv.groups = o.groups;
  s.b2.lrn.mode = o.lrn == "raw" ? LrnMode::Raw : LrnMode::DivN;
  s.d = blocks_dims(kInH, kInW, s.b1, s.b2);
  s.in_row = static_cast<size_t>(s.d.W) * s.d.C0;
  s.out_row = static_cast<size_t>(s.d.Wp2) * s.d.C2;
  if (o.init == "rand")
    init_random(s.w, s.b1, s.b2, o.seed);
  else
    init_const(s.w, s.b1, s.b2);
  if (!o.weights.empty()) {
    // raw fp32 checkpoint written by anx.utils.io.save_weights_raw (w1.bin b1.bin w2.bin b2.bin)
    auto rd = [&](const char* name, std::vector<float>& v) {
      const std::string path = o.weights + "/" + name + ".bin";
      FILE* f = std::fopen(path.c_str(), "rb");
      if (!f) throw std::runtime_error("cannot open " + path);
      const size_t got = std::fread(v.data(), sizeof(float), v.size(), f);
      const bool extra = std::fgetc(f) != EOF;
      std::fclose(f);
      if (got != v.size() || extra) throw std::runtime_error(path + ": wrong size for this configuration");
    };
    rd("w1", s.w.w1);
    rd("b1", s.w.b1);
    rd("w2", s.w.w2);
    rd("b2", s.w.b2);
  }
  return s;
}

void fill_input(Setup& s) {
  const size_t n = static_cast<size_t>(s.o.batch) * s.d.H * s.in_row;
  if (s.o.init == "rand")
    init_input_random(s.x, n, s.o.seed);
  else
    s.x.assign(n, 1.0f);
}

void bcast_weights(HostComm& c, HostWeights& w) {
  c.bcast(w.w1.data(), w.w1.size() * 4, 0);
  c.bcast(w.b1.data(), w.b1.size() * 4, 0);
  c.bcast(w.w2.data(), w.w2.size() * 4, 0);
  c.bcast(w.b2.data(), w.b2.size() * 4, 0);
}

void report(const Setup& s, int np, const std::vector<float>& y, double cold_ms, double warm_ms,
            const Phases& cold, const Phases& warm, int warm_iters, double err, const std::string& v5 = "") {
  const Options& o = s.o;
  char vals[512] = {0};
  for (int i = 0; i < 10 && i < static_cast<int>(y.size()); ++i) {
    char b[32];
    std::snprintf(b, sizeof b, "%s%g", i ? " " : "", std::round(y[i] * 1e4) / 1e4);
    std::strcat(vals, b);
  }
  const double t = warm_iters ? warm_ms : cold_ms;
  const std::string shape = std::to_string(s.d.Hp2) + "x" + std::to_string(s.d.Wp2) + "x" + std::to_string(s.d.C2);
  if (o.version == "v1") {
    const int dims[6][3] = {{s.d.H, s.d.W, s.d.C0},    {s.d.H1, s.d.W1, s.d.C1},   {s.d.Hp1, s.d.Wp1, s.d.C1},
                            {s.d.H2, s.d.W2, s.d.C2}, {s.d.Hp2, s.d.Wp2, s.d.C2}, {s.d.Hp2, s.d.Wp2, s.d.C2}};
    const char* names[6] = {"Input", "Conv1", "Pool1", "Conv2", "Pool2", "LRN2"};
    for (int i = 0; i < 6; ++i)
      std::printf("  [%s] Dimensions: H=%d, W=%d, C=%d\n", names[i], dims[i][0], dims[i][1], dims[i][2]);
    std::printf("AlexNet Serial Forward Pass completed in %.3f ms\n", t);
    std::printf("Final Output (first 10 values): %s\n", vals);
  } else if (o.version == "v2.1" || o.version == "v2.2") {
    std::printf("shape: %s\n", shape.c_str());
    std::string five(vals);
    int sp = 0;
    for (size_t i = 0; i < five.size(); ++i)
      if (five[i] == ' ' && ++sp == 5) five.resize(i);
    std::printf("Sample values: %s\n", five.c_str());
    std::printf("Execution Time: %.3f ms\n", t);
  } else if (o.version == "v3") {
    std::printf("AlexNet HIP Forward Pass completed in %.3f ms\n", t);
    std::printf("Final Output (first 10 values): %s\n", vals);
  } else {
    std::printf("Final Output Shape: %s\n", shape.c_str());
    std::printf("Final Output (first 10 values): %s\n", vals);
    std::printf("AlexNet %s+HIP Forward Pass completed in %.3f ms\n", o.version == "v5" ? "RCCL" : "MPI", t);
  }
  if (o.json) {
    std::printf(
        "ANX_JSON {\"version\": \"%s\", \"np\": %d, \"batch\": %d, \"shape\": [%d, %d, %d], \"checksum\": %u, "
        "\"cold_ms\": %.4f, \"warm_ms\": %s, \"images_per_s\": %s, \"phases_cold\": %s, \"phases_warm\": %s, "
        "\"max_abs_err\": %s, \"lrn_mode\": \"%s\", \"decomp\": \"%s\", \"impl\": \"%s\", \"native\": true%s%s}\n",
        o.version.c_str(), np, o.batch, s.d.Hp2, s.d.Wp2, s.d.C2, crc32(y.data(), y.size() * 4), cold_ms,
        warm_iters ? std::to_string(warm_ms).c_str() : "null",
        warm_iters ? std::to_string(o.batch / (warm_ms / 1e3)).c_str() : "null", cold.json().c_str(),
        warm.json(warm_iters ? 1.0 / warm_iters : 1.0).c_str(), err >= 0 ? std::to_string(err).c_str() : "null",
        o.lrn.c_str(), o.decomp.c_str(), o.impl.c_str(), v5.empty() ? "" : ", \"v5\": ", v5.c_str());
  }
  std::fflush(stdout);
}

double check_err(const Setup& s, const std::vector<float>& y) {
  std::vector<float> x = s.x;
  if (x.empty()) {
    Setup t = s;
    fill_input(t);
    x = t.x;
  }
  CpuBlocks ref(s.b1, s.b2, s.d.H, s.d.W, s.w);
  std::vector<float> r(y.size());
  ref.forward(x.data(), s.o.batch, r.data());
  double e = 0;
  for (size_t i = 0; i < y.size(); ++i) e = std::max(e, static_cast<double>(std::fabs(y[i] - r[i])));
  return e;
}

// ------------------------------------------------------------------------------ V1 / V3 (single process)
int run_single(Setup& s) {
  const int N = s.o.batch;
  Phases cold, warm;
  const double t0 = now_ms();
  fill_input(s);
  std::vector<float> y(static_cast<size_t>(N) * s.d.Hp2 * s.out_row);
  double cold_ms = 0, warm_ms = 0;
  if (s.o.version == "v1") {
    CpuBlocks eng(s.b1, s.b2, s.d.H, s.d.W, s.w);
    cold.add("setup", now_ms() - t0);
    double a = now_ms();
    eng.forward(s.x.data(), N, y.data());
    cold.add("compute", now_ms() - a);
    cold_ms = now_ms() - t0;
    for (int i = 0; i < s.o.iters; ++i) {
      a = now_ms();
      eng.forward(s.x.data(), N, y.data());
      warm.add("compute", now_ms() - a);
    }
  } else {
    // cold phases (bench.py b1_process_phases_ms): input = host init of the image, init = HIP runtime +
    // device context + stream, engine = weights (transformed / packed on the host) + workspace upload,
    // alloc = the I/O buffers; then h2d / compute / d2h of the first call
    double a0 = now_ms();
    cold.add("input", a0 - t0);
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev < 1) throw std::runtime_error("v3 needs a GPU");
    hip_check(hipSetDevice(s.ri.local_rank % ndev), "hipSetDevice");
    hipStream_t st;
    hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
    cold.add("init", now_ms() - a0);
    a0 = now_ms();
    set_upload_stream(st);  // the engine's weight uploads on this stream (the null stream's first use costs a queue)
    BlocksEngine eng(s.b1, s.b2, s.d.H, s.d.W, s.w, N, s.o.impl == "direct" ? Impl::Direct : Impl::Mfma, s.k);
    cold.add("engine", now_ms() - a0);
    a0 = now_ms();
    float *dx, *dy, *hx, *hy;
    hip_check(hipMalloc(&dx, s.x.size() * 4), "hipMalloc");
    hip_check(hipMalloc(&dy, y.size() * 4), "hipMalloc");
    // pinned I/O buffers: a copy from pageable memory would initialise the runtime's staged-copy path
    // inside the timed region (9-10 ms on its first use, anx/upload.hpp); the image is written into the
    // pinned buffer on the host, as a serving process receives it
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&hx), s.x.size() * 4, hipHostMallocDefault), "hipHostMalloc");
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&hy), y.size() * 4, hipHostMallocDefault), "hipHostMalloc");
    std::memcpy(hx, s.x.data(), s.x.size() * 4);
    cold.add("alloc", now_ms() - a0);
    auto step = [&](Phases& ph) {
      double a = now_ms();
      hip_check(hipMemcpyAsync(dx, hx, s.x.size() * 4, hipMemcpyHostToDevice, st), "H2D");
      hip_check(hipStreamSynchronize(st), "sync");
      ph.add("h2d", now_ms() - a);
      a = now_ms();
      hip_check(eng.forward(dx, N, dy, st), "forward");
      hip_check(hipStreamSynchronize(st), "sync");
      ph.add("compute", now_ms() - a);
      a = now_ms();
      hip_check(hipMemcpyAsync(hy, dy, y.size() * 4, hipMemcpyDeviceToHost, st), "D2H");
      hip_check(hipStreamSynchronize(st), "sync");
      ph.add("d2h", now_ms() - a);
    };
    step(cold);
    cold_ms = now_ms() - t0;
    for (int i = 0; i < s.o.iters; ++i) step(warm);
    std::memcpy(y.data(), hy, y.size() * 4);
    hip_check(hipFree(dx), "free");
    hip_check(hipFree(dy), "free");
    hip_check(hipHostFree(hx), "free");
    hip_check(hipHostFree(hy), "free");
    set_upload_stream(nullptr);
    hip_check(hipStreamDestroy(st), "free");
  }
  warm_ms = s.o.iters ? warm.total() / s.o.iters : 0;
  report(s, 1, y, cold_ms, warm_ms, cold, warm, s.o.iters, s.o.check ? check_err(s, y) : -1);
  return 0;
}

// ------------------------------------------------------------------------------ V2.1 (replicated)
int run_v21(Setup& s, HostComm& c) {
  const int N = s.o.batch;
  Phases cold, warm;
  c.barrier();
  const double t0 = now_ms();
  double a = now_ms();
  if (c.rank() == 0) fill_input(s);
  else s.x.resize(static_cast<size_t>(N) * s.d.H * s.in_row);
  bcast_weights(c, s.w);
  c.bcast(s.x.data(), s.x.size() * 4, 0);  // M3: the whole image to every rank (main.cpp:71)
  cold.add("bcast", now_ms() - a);
  CpuBlocks eng(s.b1, s.b2, s.d.H, s.d.W, s.w);
  std::vector<float> y(static_cast<size_t>(N) * s.d.Hp2 * s.out_row);
  auto step = [&](Phases& ph) {
    double t = now_ms();
    eng.forward(s.x.data(), N, y.data());  // every rank computes everything (P1)
    ph.add("compute", now_ms() - t);
    t = now_ms();
    c.barrier();
    ph.add("barrier", now_ms() - t);
  };
  step(cold);
  double cold_ms = now_ms() - t0;
  for (int i = 0; i < s.o.iters; ++i) step(warm);
  double tm[2] = {cold_ms, s.o.iters ? warm.total() / s.o.iters : 0};
  c.allreduce_max(tm, 2);
  if (c.rank() == 0) report(s, c.size(), y, tm[0], tm[1], cold, warm, s.o.iters, s.o.check ? check_err(s, y) : -1);
  c.barrier();
  return 0;
}

// ------------------------------------------------------------------------------ V2.2 / V4 (host-staged rows)
int run_rows_host(Setup& s, HostComm& c, bool gpu) {
  const int N = s.o.batch, rank = c.rank(), np = c.size();
  const Decomp mode = s.o.decomp == "per_layer" ? Decomp::PerLayer : Decomp::Overlap;
  const DecompPlan plan = make_plan(s.d.H, s.d.W, np, mode, s.b1, s.b2);
  const TilePlan& t = plan.tiles[rank];
  const RowRange own = plan.owned_in[rank];
  Phases cold, warm;
  c.barrier();
  const double t0 = now_ms();
  double a = now_ms();
  if (rank == 0) fill_input(s);
  bcast_weights(c, s.w);  // M4/M5
  cold.add("bcast", now_ms() - a);
  a = now_ms();
  std::unique_ptr<CpuBlocks> ceng;
  std::unique_ptr<BlocksEngine> geng;
  hipStream_t st = nullptr;
  float *d_in = nullptr, *d_y = nullptr, *h_in = nullptr, *h_y = nullptr;
  std::vector<float> tile_in(static_cast<size_t>(N) * t.in.size() * s.in_row);
  std::vector<float> y_loc(static_cast<size_t>(N) * t.out.size() * s.out_row);
  std::vector<float> own_buf(static_cast<size_t>(N) * own.size() * s.in_row);
  if (gpu) {
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev < 1) throw std::runtime_error("v4 needs a GPU");
    hip_check(hipSetDevice(s.ri.local_rank % ndev), "hipSetDevice");  // fixes reference D4
    hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
    geng = std::make_unique<BlocksEngine>(s.b1, s.b2, s.d.H, s.d.W, s.w, N,
                                          s.o.impl == "direct" ? Impl::Direct : Impl::Mfma, s.k);
    hip_check(hipMalloc(&d_in, std::max<size_t>(1, tile_in.size()) * 4), "hipMalloc");
    hip_check(hipMalloc(&d_y, std::max<size_t>(1, y_loc.size()) * 4), "hipMalloc");
    hip_check(hipHostMalloc(&h_in, std::max<size_t>(1, tile_in.size()) * 4, hipHostMallocDefault), "pinned");
    hip_check(hipHostMalloc(&h_y, std::max<size_t>(1, y_loc.size()) * 4, hipHostMallocDefault), "pinned");
  } else {
    ceng = std::make_unique<CpuBlocks>(s.b1, s.b2, s.d.H, s.d.W, s.w);
  }
  cold.add("setup", now_ms() - a);
  std::vector<float> y_full(rank == 0 ? static_cast<size_t>(N) * s.d.Hp2 * s.out_row : 0);
  std::vector<std::vector<float>> stage(np);
  std::vector<std::vector<float>> hbufs;
  // Per-layer decomposition (the reference's second exchange: V2.2 halo2 on pool1 rows, M11, and
  // V4's device-staged variant, M13): after stage1 every rank holds its own pool1 rows t.p1 in the
  // conv2 window; the rows of t.q owned by neighbours arrive over the host channel (GPU: D2H of
  // the sent rows, H2D of the received ones; a window's rows of one image are contiguous).
  std::vector<std::vector<float>> p1bufs;
  const size_t wrow = gpu ? geng->q2_row_floats() : ceng->window_row_floats();
  auto win_rows = [&](int n, int r) { return gpu ? geng->q2_row_ptr(t, n, r) : ceng->window_row(t, n, r); };
  auto p1_exchange = [&]() {
    p1bufs.clear();
    for (const HaloXfer& h : plan.p1_halos)
      if (h.src == rank || h.dst == rank) p1bufs.emplace_back(static_cast<size_t>(N) * h.rows.size() * wrow);
    size_t bi = 0;
    for (const HaloXfer& h : plan.p1_halos) {  // pack the rows this rank sends
      if (h.src != rank && h.dst != rank) continue;
      if (h.src == rank) {
        const size_t blk = h.rows.size() * wrow;
        for (int n = 0; n < N; ++n) {
          if (gpu)
            hip_check(hipMemcpyAsync(p1bufs[bi].data() + n * blk, win_rows(n, h.rows.lo), blk * 4, hipMemcpyDeviceToHost,
                                     st), "D2H halo");
          else
            std::memcpy(p1bufs[bi].data() + n * blk, win_rows(n, h.rows.lo), blk * 4);
        }
      }
      ++bi;
    }
    if (gpu) hip_check(hipStreamSynchronize(st), "sync");
    bi = 0;
    for (const HaloXfer& h : plan.p1_halos) {
      if (h.src != rank && h.dst != rank) continue;
      if (h.src == rank) c.isend(p1bufs[bi].data(), p1bufs[bi].size() * 4, h.dst);
      else c.irecv(p1bufs[bi].data(), p1bufs[bi].size() * 4, h.src);
      ++bi;
    }
    c.wait_all();
    bi = 0;
    for (const HaloXfer& h : plan.p1_halos) {  // unpack the received rows into the window
      if (h.src != rank && h.dst != rank) continue;
      if (h.dst == rank) {
        const size_t blk = h.rows.size() * wrow;
        for (int n = 0; n < N; ++n) {
          if (gpu)
            hip_check(hipMemcpyAsync(win_rows(n, h.rows.lo), p1bufs[bi].data() + n * blk, blk * 4, hipMemcpyHostToDevice,
                                     st), "H2D halo");
          else
            std::memcpy(win_rows(n, h.rows.lo), p1bufs[bi].data() + n * blk, blk * 4);
        }
      }
      ++bi;
    }
  };

  auto step = [&](Phases& ph) {
    // scatter owned input rows (Scatterv, M9)
    double q = now_ms();
    roctx_push("v4 scatter");
    if (rank == 0) {
      for (int r = 0; r < np; ++r) {
        const RowRange o = plan.owned_in[r];
        if (o.empty()) continue;
        float* dst = r == 0 ? own_buf.data() : (stage[r].resize(static_cast<size_t>(N) * o.size() * s.in_row),
                                               stage[r].data());
        copy_rows(dst, o.size(), 0, s.x.data(), s.d.H, o.lo, o.size(), s.in_row, N, false, nullptr);
        if (r) c.isend(dst, stage[r].size() * 4, r);
      }
    } else if (!own.empty()) {
      c.irecv(own_buf.data(), own_buf.size() * 4, 0);
    }
    c.wait_all();
    roctx_pop();
    ph.add("scatter", now_ms() - q);
    // input halo exchange (M10/M12) — planner transfers, both directions in one group
    q = now_ms();
    roctx_push("v4 halo_in");
    hbufs.clear();
    std::vector<std::pair<RowRange, float*>> recvs;
    for (const HaloXfer& h : plan.in_halos) {
      if (h.src == rank) {
        hbufs.emplace_back(static_cast<size_t>(N) * h.rows.size() * s.in_row);
        copy_rows(hbufs.back().data(), h.rows.size(), 0, own_buf.data(), own.size(), h.rows.lo - own.lo,
                  h.rows.size(), s.in_row, N, false, nullptr);
      } else if (h.dst == rank) {
        hbufs.emplace_back(static_cast<size_t>(N) * h.rows.size() * s.in_row);
      }
    }
    size_t bi = 0;
    for (const HaloXfer& h : plan.in_halos) {
      if (h.src == rank) c.isend(hbufs[bi++].data(), static_cast<size_t>(N) * h.rows.size() * s.in_row * 4, h.dst);
      else if (h.dst == rank) {
        c.irecv(hbufs[bi].data(), static_cast<size_t>(N) * h.rows.size() * s.in_row * 4, h.src);
        recvs.push_back({h.rows, hbufs[bi++].data()});
      }
    }
    c.wait_all();
    if (!t.out.empty()) {
      const int lo = std::max(own.lo, t.in.lo), hi = std::min(own.hi, t.in.hi);
      copy_rows(tile_in.data(), t.in.size(), lo - t.in.lo, own_buf.data(), own.size(), lo - own.lo, hi - lo,
                s.in_row, N, false, nullptr);
      for (auto& rv : recvs)
        copy_rows(tile_in.data(), t.in.size(), rv.first.lo - t.in.lo, rv.second, rv.first.size(), 0,
                  rv.first.size(), s.in_row, N, false, nullptr);
    }
    roctx_pop();
    ph.add("halo", now_ms() - q);
    // compute (V4: host -> device -> host around the tile, pinned buffers)
    if (!t.out.empty()) {
      if (gpu) {
        RoctxRange rc("v4 h2d+compute+d2h");
        q = now_ms();
        std::memcpy(h_in, tile_in.data(), tile_in.size() * 4);
        hip_check(hipMemcpyAsync(d_in, h_in, tile_in.size() * 4, hipMemcpyHostToDevice, st), "H2D");
        hip_check(hipStreamSynchronize(st), "sync");
        ph.add("h2d", now_ms() - q);
        q = now_ms();
        if (mode == Decomp::Overlap) {
          hip_check(geng->tile_forward(d_in, N, t, d_y, st), "tile_forward");
        } else {
          hip_check(geng->stage1(d_in, N, t, st), "stage1");
          hip_check(hipStreamSynchronize(st), "sync");
          ph.add("compute", now_ms() - q);
          q = now_ms();
          {
            RoctxRange rh("v4 halo_p1");
            p1_exchange();
          }
          ph.add("halo_p1", now_ms() - q);
          q = now_ms();
          hip_check(geng->stage2(N, t, d_y, st), "stage2");
        }
        hip_check(hipStreamSynchronize(st), "sync");
        ph.add("compute", now_ms() - q);
        q = now_ms();
        hip_check(hipMemcpyAsync(h_y, d_y, y_loc.size() * 4, hipMemcpyDeviceToHost, st), "D2H");
        hip_check(hipStreamSynchronize(st), "sync");
        std::memcpy(y_loc.data(), h_y, y_loc.size() * 4);
        ph.add("d2h", now_ms() - q);
      } else {
        q = now_ms();
        if (mode == Decomp::Overlap) {
          ceng->tile_forward(tile_in.data(), N, t, y_loc.data());
        } else {
          ceng->stage1(tile_in.data(), N, t);
          ph.add("compute", now_ms() - q);
          q = now_ms();
          {
            RoctxRange rh("v2.2 halo_p1");
            p1_exchange();
          }
          ph.add("halo_p1", now_ms() - q);
          q = now_ms();
          ceng->stage2(N, t, y_loc.data());
        }
        ph.add("compute", now_ms() - q);
      }
    }
    // gather output rows (Gatherv, M16)
    q = now_ms();
    RoctxRange rg("v4 gather");
    if (rank == 0) {
      for (int r = 1; r < np; ++r) {
        const RowRange o = plan.tiles[r].out;
        if (o.empty()) continue;
        stage[r].resize(static_cast<size_t>(N) * o.size() * s.out_row);
        c.irecv(stage[r].data(), stage[r].size() * 4, r);
      }
      c.wait_all();
      for (int r = 0; r < np; ++r) {
        const RowRange o = plan.tiles[r].out;
        if (o.empty()) continue;
        copy_rows(y_full.data(), s.d.Hp2, o.lo, r == 0 ? y_loc.data() : stage[r].data(), o.size(), 0, o.size(),
                  s.out_row, N, false, nullptr);
      }
    } else if (!t.out.empty()) {
      c.send(y_loc.data(), y_loc.size() * 4, 0);
    }
    ph.add("gather", now_ms() - q);
  };
  step(cold);
  double cold_ms = now_ms() - t0;
  for (int i = 0; i < s.o.iters; ++i) step(warm);
  double tm[2] = {cold_ms, s.o.iters ? warm.total() / s.o.iters : 0};
  c.allreduce_max(tm, 2);
  if (rank == 0) report(s, np, y_full, tm[0], tm[1], cold, warm, s.o.iters, s.o.check ? check_err(s, y_full) : -1);
  if (gpu) {
    (void)hipFree(d_in);
    (void)hipFree(d_y);
    (void)hipHostFree(h_in);
    (void)hipHostFree(h_y);
    (void)hipStreamDestroy(st);
  }
  c.barrier();
  return 0;
}

// ------------------------------------------------------------------------------ V5 (device-resident)
// The V5 runtime (anx/v5.hpp): one transfer schedule per step (with --input-source root a scatter of
// images x input rows; pool1 halos inside each row group cut into image chunks that move while stage1
// computes the next chunk; gather of output rows), executed by a pluggable transport:
//   rccl      grouped ncclSend/ncclRecv over xGMI (one GPU per rank),
//   loopback  the same RCCL transport code over the loopback device comm (ranks share a GPU),
//   peer      one hipMemcpy2DAsync per transfer into the receiver's IPC-mapped buffer, ordered by
//             device-side flags (ranks may share a GPU: the configuration the one-GPU test box can run).
// Steady-state steps never synchronise a stream with the host. Phase times are the compute stream's
// critical path (scatter / halo_p1 = time spent waiting for data). --dry-run prints the schedule each
// rank's transport would execute (record-only, no GPU) as ANX_SCHEDULE lines.
int run_v5_steps(Setup& s, HostComm& c, V5Runtime& rt, int N, double t0);

int run_v5(Setup& s, HostComm& c, bool dry) {
  const int N = s.o.batch, rank = c.rank(), np = c.size();
  V5Options o;
  o.batch = N;
  o.row_ways = s.o.split == "rows" ? np : s.o.split == "hybrid" ? 0 : s.o.split == "batch" ? 1 : -1;
  if (s.o.row_ways > 0) {
    if (np % s.o.row_ways) throw std::invalid_argument("--row-ways must divide the rank count");
    o.row_ways = s.o.row_ways;
  }
  o.mode = s.o.decomp == "overlap" ? Decomp::Overlap : Decomp::PerLayer;
  o.transport = s.o.transport;
  o.chunks = s.o.chunks;
  o.pipeline = s.o.pipeline == "on" ? 1 : s.o.pipeline == "off" ? 0 : -1;
  o.poison = s.o.poison;
  o.impl = s.o.impl == "direct" ? Impl::Direct : Impl::Mfma;
  o.knobs = s.k;
  o.peer_sync = s.o.peer_sync;
  o.input_source = s.o.input_source == "root" ? InputSource::Root : InputSource::Local;
  if (s.o.lanes > 0) o.lanes = s.o.lanes;
  if (dry) {  // the schedule this rank's transport would execute, one step
    const std::string tr = pick_v5_transport(o.transport, s.ri, 0, true);
    const std::vector<std::string> log = v5_dry_schedule(rank, np, s.b1, s.b2, s.d.H, s.d.W, o, tr);
    for (int r = 0; r < np; ++r) {
      if (r == rank)
        for (const std::string& l : log) std::printf("ANX_SCHEDULE %s rank %d: %s\n", tr.c_str(), rank, l.c_str());
      std::fflush(stdout);
      c.barrier();
    }
    return 0;
  }
  c.barrier();
  const double t0 = now_ms();
  if (rank == 0) fill_input(s);
  V5Runtime rt(c, s.ri, s.b1, s.b2, s.d.H, s.d.W, s.w, o);
  try {
    return run_v5_steps(s, c, rt, N, t0);
  } catch (...) {
    rt.abort();  // before ~V5Runtime's device sync: release every wait on a peer (ncclCommAbort / flags)
    throw;
  }
}

// The timed part of run_v5 (t0: its start, before the runtime's construction).
int run_v5_steps(Setup& s, HostComm& c, V5Runtime& rt, int N, double t0) {
  const int rank = c.rank(), np = c.size();
  Phases cold, warm;
  rt.set_input(rank == 0 ? s.x.data() : nullptr);
  const double a = t0;
  cold.add("setup", now_ms() - a);
  std::vector<float> y_host(rank == 0 ? static_cast<size_t>(N) * s.d.Hp2 * s.out_row : 0);
  rt.step();
  rt.sync();
  for (const auto& kv : rt.phase_ms()) cold.add(kv.first, kv.second);
  rt.reset_phases();
  if (rank == 0) rt.output(y_host.data());
  const double cold_ms = now_ms() - t0;
  double wall = 0;
  if (s.o.iters > 0) {
    c.barrier();
    const double w0 = now_ms();
    for (int i = 0; i < s.o.iters; ++i) rt.step();  // no host sync inside
    rt.sync();
    c.barrier();
    wall = (now_ms() - w0) / s.o.iters;
    for (const auto& kv : rt.phase_ms()) warm.add(kv.first, kv.second * s.o.iters);
    if (rank == 0) rt.output(y_host.data());
  }
  double tm[2] = {cold_ms, wall};
  c.allreduce_max(tm, 2);
  if (rank == 0) {
    std::printf("ANX_TRANSPORT %s ordering %s\n", rt.transport(), rt.pipelined() ? "pipelined" : "serial");
    report(s, np, y_host, tm[0], tm[1], cold, warm, s.o.iters, s.o.check ? check_err(s, y_host) : -1,
           rt.describe_json());
  }
  return 0;  // ~V5Runtime: collective teardown
}

}  // namespace

int main(int argc, char** argv) {
  const Options o = parse(argc, argv);
  const RankInfo ri = rank_info_from_env();
  // V3 is a one-image latency program: its copies (2.6 MB of weights, the image, the output) are small,
  // and the runtime's first SDMA copy of a process brings the engine queue up (~8 ms on an MI355X box for
  // any copy >= 64 KiB; 0.35 ms for 2.5 MiB through the blit kernels instead, anx_hipinit,
  // profiles/r06_cold/). Read by the runtime at its first call, so set before anything touches HIP; an
  // explicit HSA_ENABLE_SDMA in the environment wins. The multi-rank versions keep SDMA for their
  // large per-step transfers.
  if (o.version == "v3") setenv("HSA_ENABLE_SDMA", "0", 0);
  try {
    Setup s = make_setup(o, ri);
    if (o.version == "v1" || o.version == "v3") {
      if (ri.world > 1) throw std::runtime_error(o.version + " is a single-process version");
      return run_single(s);
    }
    const char* tmo = std::getenv("ANX_COMM_TIMEOUT");
    HostComm c(ri, tmo ? std::atof(tmo) : 300.0);
    // Fault injection for the fail-stop tests: ANX_FAULT=exit:R | hang:R makes rank R
    // exit(3) or stall after bootstrap; the peers must abort (comm watchdog / closed sockets).
    if (const char* f = std::getenv("ANX_FAULT")) {
      const std::string fs(f);
      const size_t colon = fs.find(':');
      if (colon != std::string::npos && std::atoi(fs.c_str() + colon + 1) == ri.rank) {
        if (fs.compare(0, colon, "exit") == 0) c.abort("injected fault (exit)", 3);
        if (fs.compare(0, colon, "hang") == 0)
          for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
      }
    }
    try {
      if (o.version == "v2.1") return run_v21(s, c);
      if (o.version == "v2.2") return run_rows_host(s, c, false);
      if (o.version == "v4") return run_rows_host(s, c, true);
      return run_v5(s, c, o.dry_run);
    } catch (const std::exception& e) {
      c.abort(e.what());  // coordinated fail-stop (the reference's CUDA_CHECK -> MPI_Abort, N29)
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[anx rank %d] error: %s\n", ri.rank, e.what());
    return 1;
  }
}
