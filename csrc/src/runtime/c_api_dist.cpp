// C ABI of the multi-GPU runtimes (anx/c_api.h, "V4 / V5 multi-GPU runtimes"): libanx_dist.so, loaded
// by anx._native.dist() for bench.py --workload v4|v5 and anx.parallel.workloads.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>

#include "anx/c_api.h"
#include "anx/v4.hpp"
#include "anx/v5.hpp"

namespace {

struct V5Handle {
  std::unique_ptr<anx::HostComm> comm;
  std::unique_ptr<anx::V5Runtime> rt;  // destroyed first (its teardown is collective over comm)
};

template <class F>
int guarded(const char* what, F&& f) {
  try {
    return f();
  } catch (const std::exception& ex) {
    anx_set_last_error((std::string(what) + ": " + ex.what()).c_str());
  } catch (...) {
    anx_set_last_error((std::string(what) + ": unknown exception").c_str());
  }
  return 1;
}

anx::BlockSpec spec(const anx_block_c& b) {
  anx::BlockSpec s{};
  s.conv = {b.C, b.K, b.F, b.S, b.P, b.groups};
  s.pool = {b.pool_F, b.pool_S};
  s.has_lrn = b.has_lrn != 0;
  s.lrn = {b.lrn_N, b.lrn_alpha, b.lrn_beta, b.lrn_k, static_cast<anx::LrnMode>(b.lrn_mode)};
  return s;
}

int put(const std::string& s, char* buf, size_t cap) {
  if (!buf || cap == 0) return 0;
  const size_t n = std::min(s.size(), cap - 1);
  std::memcpy(buf, s.data(), n);
  buf[n] = 0;
  if (s.size() >= cap) {
    anx_set_last_error("output buffer too small");
    return 2;
  }
  return 0;
}

anx::V5Options options(int batch, int row_ways, int mode, const char* transport, int chunks, int input_source) {
  anx::V5Options o;
  o.batch = batch;
  o.row_ways = row_ways;
  o.mode = mode ? anx::Decomp::PerLayer : anx::Decomp::Overlap;
  o.transport = transport ? transport : "auto";
  o.chunks = chunks;
  o.input_source = input_source ? anx::InputSource::Root : anx::InputSource::Local;
  return o;
}

struct V4Handle {
  std::unique_ptr<anx::HostComm> comm;
  std::unique_ptr<anx::V4Runtime> rt;
};
V4Handle* H4(void* h) {
  if (!h) throw std::invalid_argument("null v4 handle");
  return static_cast<V4Handle*>(h);
}

anx::RankInfo rank_info(int rank, int world, int local_rank, int local_world, int nnodes, const char* master_addr,
                        int master_port) {
  anx::RankInfo ri;
  ri.rank = rank;
  ri.world = world;
  ri.local_rank = local_rank;
  ri.local_world = local_world;
  ri.nnodes = nnodes;
  ri.master_addr = master_addr ? master_addr : "127.0.0.1";
  ri.master_port = master_port;
  return ri;
}

anx::HostWeights root_weights(int rank, const anx::BlockSpec& s1, const anx::BlockSpec& s2, const float* w1,
                              const float* bias1, const float* w2, const float* bias2) {
  anx::HostWeights w;
  if (rank == 0) {
    if (!w1 || !bias1 || !w2 || !bias2) throw std::invalid_argument("rank 0 needs the weights");
    anx::init_const(w, s1, s2);
    std::memcpy(w.w1.data(), w1, w.w1.size() * 4);
    std::memcpy(w.b1.data(), bias1, w.b1.size() * 4);
    std::memcpy(w.w2.data(), w2, w.w2.size() * 4);
    std::memcpy(w.b2.data(), bias2, w.b2.size() * 4);
  }
  return w;
}

std::string phases_json(const std::vector<std::pair<std::string, double>>& v) {
  std::string s = "{";
  char b[96];
  for (size_t i = 0; i < v.size(); ++i) {
    std::snprintf(b, sizeof b, "%s\"%s\": %.5f", i ? ", " : "", v[i].first.c_str(), v[i].second);
    s += b;
  }
  return s + "}";
}

V5Handle* H(void* h) {
  if (!h) throw std::invalid_argument("null v5 handle");
  return static_cast<V5Handle*>(h);
}

}  // namespace

extern "C" {

int anx_v5_create(void** out, int rank, int world, int local_rank, int local_world, int nnodes,
                  const char* master_addr, int master_port, double timeout_s, const anx_block_c* b1,
                  const anx_block_c* b2, int H, int W, const float* w1, const float* bias1, const float* w2,
                  const float* bias2, int batch, int row_ways, int mode, const char* transport, int chunks,
                  int pipeline, int poison, int impl, const char* peer_sync, int input_source, int lanes,
                  int keep_log, int root_images) {
  return guarded("anx_v5_create", [&] {
    if (!out || !b1 || !b2) throw std::invalid_argument("null argument");
    const anx::RankInfo ri = rank_info(rank, world, local_rank, local_world, nnodes, master_addr, master_port);
    anx::V5Options o = options(batch, row_ways, mode, transport, chunks, input_source);
    o.lanes = lanes > 0 ? lanes : o.lanes;
    o.keep_log = keep_log != 0;
    o.root_images = root_images;
    o.pipeline = pipeline;
    o.poison = poison != 0;
    o.impl = impl == 1 ? anx::Impl::Direct : anx::Impl::Mfma;
    o.host = impl == 2;  // CPU ranks: the host engine and the host transport, no HIP call
    o.peer_sync = peer_sync ? peer_sync : "";
    const anx::BlockSpec s1 = spec(*b1), s2 = spec(*b2);
    const anx::HostWeights w = root_weights(rank, s1, s2, w1, bias1, w2, bias2);
    auto h = std::make_unique<V5Handle>();
    h->comm = std::make_unique<anx::HostComm>(ri, timeout_s > 0 ? timeout_s : 300.0);
    h->rt = std::make_unique<anx::V5Runtime>(*h->comm, ri, s1, s2, H, W, w, o);
    *out = h.release();
    return 0;
  });
}

int anx_v5_destroy(void* h) {
  return guarded("anx_v5_destroy", [&] {
    std::unique_ptr<V5Handle> p(static_cast<V5Handle*>(h));
    if (p) p->rt.reset();
    return 0;
  });
}

int anx_v5_set_input(void* h, const float* host_x) {
  return guarded("anx_v5_set_input", [&] {
    H(h)->rt->set_input(host_x);
    return 0;
  });
}

int anx_v5_step(void* h, int steps) {
  return guarded("anx_v5_step", [&] {
    try {
      for (int i = 0; i < steps; ++i) H(h)->rt->step();
    } catch (...) {
      H(h)->rt->abort();  // fail-stop: no stream of this rank stays parked on a peer
      throw;
    }
    return 0;
  });
}

int anx_v5_sync(void* h) {
  return guarded("anx_v5_sync", [&] {
    try {
      H(h)->rt->sync();
    } catch (...) {
      H(h)->rt->abort();
      throw;
    }
    return 0;
  });
}

int anx_v5_output(void* h, float* host_y) {
  return guarded("anx_v5_output", [&] {
    H(h)->rt->output(host_y);
    return 0;
  });
}

int anx_v5_phases(void* h, char* buf, size_t cap, int reset) {
  return guarded("anx_v5_phases", [&] {
    anx::V5Runtime& rt = *H(h)->rt;
    const std::string s = phases_json(rt.phase_ms());
    if (reset) rt.reset_phases();
    return put(s, buf, cap);
  });
}

int anx_v5_describe(void* h, char* buf, size_t cap) {
  return guarded("anx_v5_describe", [&] { return put(H(h)->rt->describe_json(), buf, cap); });
}

int anx_v5_log(void* h, char* buf, size_t cap) {
  return guarded("anx_v5_log", [&] {
    std::string s;
    for (const std::string& l : H(h)->rt->transfer_log()) s += l + "\n";
    return put(s, buf, cap);
  });
}

int anx_v5_schedule(int np, const anx_block_c* b1, const anx_block_c* b2, int H, int W, int batch, int row_ways,
                    int mode, int chunks, int rank, const char* transport, int input_source, char* buf, size_t cap) {
  return guarded("anx_v5_schedule", [&] {
    if (!b1 || !b2) throw std::invalid_argument("null block spec");
    const anx::V5Options o = options(batch, row_ways, mode, transport, chunks, input_source);
    std::string s;
    if (rank < 0) {
      for (const anx::Transfer& x : anx::make_v5_layout(np, spec(*b1), spec(*b2), H, W, o).step_transfers())
        s += x.str() + "\n";
    } else {
      const std::string tr = transport ? transport : "rccl";
      for (const std::string& l : anx::v5_dry_schedule(rank, np, spec(*b1), spec(*b2), H, W, o, tr)) s += l + "\n";
    }
    return put(s, buf, cap);
  });
}

// ---------------------------------------------------------------------------------------------- V4
int anx_v4_create(void** out, int rank, int world, int local_rank, int local_world, int nnodes,
                  const char* master_addr, int master_port, double timeout_s, const anx_block_c* b1,
                  const anx_block_c* b2, int H, int W, const float* w1, const float* bias1, const float* w2,
                  const float* bias2, int batch, int row_ways, int chunks, int impl) {
  return guarded("anx_v4_create", [&] {
    if (!out || !b1 || !b2) throw std::invalid_argument("null argument");
    const anx::RankInfo ri = rank_info(rank, world, local_rank, local_world, nnodes, master_addr, master_port);
    anx::V4Options o;
    o.batch = batch;
    o.row_ways = row_ways;
    o.chunks = chunks;
    o.impl = impl ? anx::Impl::Direct : anx::Impl::Mfma;
    const anx::BlockSpec s1 = spec(*b1), s2 = spec(*b2);
    const anx::HostWeights w = root_weights(rank, s1, s2, w1, bias1, w2, bias2);
    auto h = std::make_unique<V4Handle>();
    h->comm = std::make_unique<anx::HostComm>(ri, timeout_s > 0 ? timeout_s : 300.0);
    h->rt = std::make_unique<anx::V4Runtime>(*h->comm, ri, s1, s2, H, W, w, o);
    *out = h.release();
    return 0;
  });
}

int anx_v4_destroy(void* h) {
  return guarded("anx_v4_destroy", [&] {
    std::unique_ptr<V4Handle> p(static_cast<V4Handle*>(h));
    if (p) p->rt.reset();
    return 0;
  });
}

int anx_v4_segment(void* h, float** input, const float** output) {
  return guarded("anx_v4_segment", [&] {
    if (input) *input = H4(h)->rt->host_input();
    if (output) *output = H4(h)->rt->host_output();
    return 0;
  });
}

int anx_v4_input_ready(void* h) {
  return guarded("anx_v4_input_ready", [&] {
    H4(h)->rt->input_ready();
    return 0;
  });
}

int anx_v4_step(void* h, int steps) {
  return guarded("anx_v4_step", [&] {
    for (int i = 0; i < steps; ++i) H4(h)->rt->step();
    return 0;
  });
}

int anx_v4_sync_all(void* h) {
  return guarded("anx_v4_sync_all", [&] {
    H4(h)->rt->sync_all();
    return 0;
  });
}

int anx_v4_phases(void* h, char* buf, size_t cap, int reset) {
  return guarded("anx_v4_phases", [&] {
    anx::V4Runtime& rt = *H4(h)->rt;
    const std::string s = phases_json(rt.phase_ms());
    if (reset) rt.reset_phases();
    return put(s, buf, cap);
  });
}

int anx_v4_probe_h2d(void* h, int reps, double* gbps) {
  return guarded("anx_v4_probe_h2d", [&] {
    *gbps = H4(h)->rt->probe_h2d_gbps(reps);
    return 0;
  });
}

int anx_v4_describe(void* h, char* buf, size_t cap) {
  return guarded("anx_v4_describe", [&] { return put(H4(h)->rt->describe_json(), buf, cap); });
}

}  // extern "C"
