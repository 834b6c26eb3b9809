// Step-time cost model of the multi-GPU workloads (anx/cost.hpp).
#include "anx/cost.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <stdexcept>

namespace anx {

namespace {

// images/s of one GPU running `imgs` whole-image equivalents per step: log2-linear between the
// measured points, flat outside them
double rate_at(const CostParams& p, double imgs) {
  const size_t n = std::min(p.rate_images.size(), p.rate_img_s.size());
  if (n == 0) throw std::invalid_argument("cost model: empty rate table");
  if (imgs <= p.rate_images[0]) return p.rate_img_s[0];
  for (size_t i = 1; i < n; ++i)
    if (imgs <= p.rate_images[i]) {
      const double a = std::log2(static_cast<double>(p.rate_images[i - 1])), b = std::log2(static_cast<double>(p.rate_images[i]));
      const double t = (std::log2(imgs) - a) / (b - a);
      return p.rate_img_s[i - 1] + t * (p.rate_img_s[i] - p.rate_img_s[i - 1]);
    }
  return p.rate_img_s[n - 1];
}

double num(const std::string& v, const std::string& what) {
  size_t used = 0;
  double x = 0;
  try {
    x = std::stod(v, &used);
  } catch (const std::exception&) {
    used = 0;
  }
  if (used == 0 || used != v.size()) throw std::invalid_argument("cost model: bad value for " + what + ": '" + v + "'");
  return x;
}

const char* wl_name(Workload w) { return w == Workload::DP ? "dp" : w == Workload::V4 ? "v4" : "v5"; }

}  // namespace

std::string StepCost::json() const {
  char b[1600];
  std::snprintf(
      b, sizeof b,
      "{\"workload\": \"%s\", \"np\": %d, \"batch\": %d, \"row_ways\": %d, \"groups\": %d, \"input_source\": \"%s\", "
      "\"decomp\": \"%s\", \"step_ms\": %.4f, \"images_per_s\": %.1f, \"bound\": \"%s\", \"compute_ms\": %.4f, "
      "\"egress_ms\": %.4f, \"ingress_ms\": %.4f, \"halo_ms\": %.4f, \"halo_exposed_ms\": %.4f, \"h2d_ms\": %.4f, "
      "\"d2h_ms\": %.4f, \"bytes\": {\"root_egress\": %.0f, \"root_ingress\": %.0f, \"max_peer_egress\": %.0f, "
      "\"max_peer_ingress\": %.0f, \"max_rank_h2d\": %.0f, \"max_rank_d2h\": %.0f, \"total_h2d\": %.0f, "
      "\"max_rank_halo\": %.0f}, \"max_rank_work_images\": %.3f, \"root_batch\": %d, \"images\": %d}",
      wl_name(wl), np, batch, row_ways, groups, src == InputSource::Local ? "local" : "root",
      mode == Decomp::PerLayer ? "per_layer" : "overlap", step_ms, images_per_s, bound.c_str(), compute_ms, egress_ms,
      ingress_ms, halo_ms, halo_exposed_ms, h2d_ms, d2h_ms, root_egress_bytes, root_ingress_bytes, max_peer_egress_bytes,
      max_peer_ingress_bytes, max_rank_h2d_bytes, max_rank_d2h_bytes, total_h2d_bytes, max_rank_halo_bytes,
      max_rank_work, root_batch, images);
  return b;
}

CostParams cost_params(const std::string& overrides) {
  CostParams p;
  size_t i = 0;
  while (i < overrides.size()) {
    size_t j = overrides.find(';', i);
    if (j == std::string::npos) j = overrides.size();
    const std::string kv = overrides.substr(i, j - i);
    i = j + 1;
    if (kv.empty()) continue;
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) throw std::invalid_argument("cost model: expected name=value, got '" + kv + "'");
    const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    if (k == "rate") {
      p.rate_images.clear();
      p.rate_img_s.clear();
      size_t a = 0;
      while (a < v.size()) {
        size_t b = v.find(',', a);
        if (b == std::string::npos) b = v.size();
        const std::string pt = v.substr(a, b - a);
        const size_t c = pt.find(':');
        if (c == std::string::npos) throw std::invalid_argument("cost model: rate points are IMAGES:IMG_PER_S");
        const int imgs = static_cast<int>(num(pt.substr(0, c), "rate"));
        if (imgs < 1 || (!p.rate_images.empty() && imgs <= p.rate_images.back()))
          throw std::invalid_argument("cost model: rate images must increase");
        p.rate_images.push_back(imgs);
        p.rate_img_s.push_back(num(pt.substr(c + 1), "rate"));
        a = b + 1;
      }
      if (p.rate_images.empty()) throw std::invalid_argument("cost model: empty rate table");
      continue;
    }
    const double x = num(v, k);
    if (k == "stage1_share") p.stage1_share = x;
    else if (k == "split_penalty") p.split_penalty = x;
    else if (k == "xgmi_gbps") p.xgmi_gbps = x;
    else if (k == "h2d_gbps") p.h2d_gbps = x;
    else if (k == "d2h_gbps") p.d2h_gbps = x;
    else if (k == "host_gbps") p.host_gbps = x;
    else if (k == "ingest_slowdown") p.ingest_slowdown = x;
    else if (k == "phase_latency_ms") p.phase_latency_ms = x;
    else if (k == "min_step_ms") p.min_step_ms = x;
    else if (k == "dp_root_shed") p.dp_root_shed = static_cast<int>(x);
    else if (k == "v4_fill") p.v4_fill = x;
    else if (k == "v5_chunks") p.v5_chunks = static_cast<int>(x);
    else throw std::invalid_argument("cost model: unknown parameter '" + k + "'");
  }
  if (p.xgmi_gbps <= 0 || p.h2d_gbps <= 0 || p.d2h_gbps <= 0 || p.host_gbps <= 0)
    throw std::invalid_argument("cost model: link rates must be positive");
  return p;
}

namespace {
constexpr double kProbeBytes = 155.06e6;  // the probe's receive volume per step (7 x 128 x 173,056 B)
double root_slowdown(const CostParams& p, double ingress_bytes) { return p.ingest_slowdown * ingress_bytes / kProbeBytes; }
}  // namespace

int dp_root_batch(int np, int batch, const CostParams& p, int H, int W) {
  if (np <= 1 || !p.dp_root_shed) return batch;
  const BlocksDims d = blocks_dims(H, W);
  const double ingress = static_cast<double>(np - 1) * batch * d.Hp2 * d.Wp2 * d.C2 * 4;
  const int b0 = 2 * static_cast<int>(std::lround(batch / (1 + root_slowdown(p, ingress)) / 2));
  return std::min(batch, std::max(2, b0));  // never above the batch (batch 1 stays 1)
}

StepCost model_step(Workload wl, int np, int batch, int row_ways, InputSource src, Decomp mode, const CostParams& p,
                    const BlockSpec& b1, const BlockSpec& b2, int H, int W) {
  if (row_ways < 0) row_ways = pick_row_ways(wl, np, batch, src, mode, p, b1, b2, H, W);
  StepCost c;
  c.wl = wl;
  c.np = np;
  c.batch = batch;
  c.src = src;
  // dp is a pure batch split of np x batch images; V4 runs overlap tiles (no mid-network exchange)
  if (wl == Workload::DP) row_ways = 1, mode = Decomp::Overlap;
  if (wl == Workload::V4) mode = Decomp::Overlap;
  c.mode = mode;
  c.row_ways = row_ways;
  const int root_b = wl == Workload::DP ? dp_root_batch(np, batch, p, H, W) : batch;
  const int global = wl == Workload::DP ? np * batch : batch;
  HybridPlan hp;
  if (!make_hybrid_plan(H, W, np, global, row_ways, mode, hp, b1, b2))
    throw std::invalid_argument("cost model: invalid plan (row_ways " + std::to_string(row_ways) + " over " +
                                std::to_string(np) + " ranks)");
  c.groups = hp.groups;
  const BlocksDims d = blocks_dims(H, W, b1, b2);
  const double in_row = static_cast<double>(d.W) * d.C0 * 4, out_row = static_cast<double>(d.Wp2) * d.C2 * 4;
  const double win_row = static_cast<double>(d.Wp1 + 2 * b2.conv.P) * d.C1 * 4;

  // per-rank compute, scatter, gather and host bytes
  double compute_max = 0, root_compute = 0;
  for (int r = 0; r < np; ++r) {
    const TilePlan& t = hp.tile(r);
    int n = t.out.empty() ? 0 : hp.images[hp.group_of[r]].size();
    if (wl == Workload::DP && r == 0) n = root_b;  // the root's shed share
    if (r == 0) c.root_batch = n;
    c.images += n;
    if (n == 0) continue;
    const bool whole = t.in.size() == H && t.out.size() == d.Hp2;
    const double eq = n * (p.stage1_share * t.c1.size() / d.H1 + (1 - p.stage1_share) * t.c2.size() / d.H2);
    double ms = std::max(p.min_step_ms, eq / rate_at(p, eq) * 1e3);
    if (!whole && mode == Decomp::PerLayer) ms *= p.split_penalty;
    if (r == 0) root_compute = ms;
    compute_max = std::max(compute_max, ms);
    c.max_rank_work = std::max(c.max_rank_work, eq);
    const double in_b = static_cast<double>(n) * t.in.size() * in_row, out_b = static_cast<double>(n) * t.out.size() * out_row;
    if (wl == Workload::V4) {
      c.max_rank_h2d_bytes = std::max(c.max_rank_h2d_bytes, in_b);
      c.max_rank_d2h_bytes = std::max(c.max_rank_d2h_bytes, out_b);
      c.total_h2d_bytes += in_b;
    } else if (r != 0) {
      if (src == InputSource::Root) {
        c.root_egress_bytes += in_b;
        c.max_peer_egress_bytes = std::max(c.max_peer_egress_bytes, in_b);
      }
      c.root_ingress_bytes += out_b;
      c.max_peer_ingress_bytes = std::max(c.max_peer_ingress_bytes, out_b);
    }
  }
  // per-layer pool1 halos: bytes each rank sends and receives (its busier direction)
  if (wl == Workload::V5 && mode == Decomp::PerLayer) {
    std::vector<double> sent(np, 0), recv(np, 0);
    int base = 0;
    for (int g = 0; g < hp.groups; ++g) {
      const int n = hp.images[g].size();
      for (const HaloXfer& h : hp.row_plans[g].p1_halos) {
        const double b = static_cast<double>(n) * h.rows.size() * win_row;
        sent[base + h.src] += b;
        recv[base + h.dst] += b;
      }
      base += hp.group_size[g];
    }
    for (int r = 0; r < np; ++r) c.max_rank_halo_bytes = std::max({c.max_rank_halo_bytes, sent[r], recv[r]});
  }

  const double link = p.xgmi_gbps * 1e6;  // bytes per ms
  c.compute_ms = compute_max;
  c.egress_ms = c.max_peer_egress_bytes / link;
  c.ingress_ms = c.max_peer_ingress_bytes / link;
  if (np > 1 && c.root_ingress_bytes > 0)  // the root computes while its links receive the gather
    c.compute_ms = std::max(compute_max, root_compute * (1 + root_slowdown(p, c.root_ingress_bytes)));
  if (wl == Workload::V4) {
    c.h2d_ms = std::max(c.max_rank_h2d_bytes / (p.h2d_gbps * 1e6), c.total_h2d_bytes / (p.host_gbps * 1e6));
    c.d2h_ms = c.max_rank_d2h_bytes / (p.d2h_gbps * 1e6);
    const double stages[3] = {c.h2d_ms, c.compute_ms, c.d2h_ms};
    const double mx = *std::max_element(stages, stages + 3), sum = stages[0] + stages[1] + stages[2];
    c.step_ms = mx + (sum - mx) * p.v4_fill;
    c.bound = mx == c.compute_ms ? "compute"
              : mx == c.d2h_ms   ? "d2h"
              : c.h2d_ms == c.total_h2d_bytes / (p.host_gbps * 1e6) ? "host"
                                                                    : "h2d";
  } else {
    if (c.max_rank_halo_bytes > 0) {
      int chunks = p.v5_chunks;
      if (chunks <= 0) chunks = 1;  // the runtime's auto rule (make_v5_layout): one chunk
      c.halo_ms = c.max_rank_halo_bytes / link;
      c.halo_exposed_ms = c.halo_ms / chunks + p.phase_latency_ms * chunks;
    }
    const double io = c.egress_ms + c.ingress_ms + (np > 1 ? p.phase_latency_ms * (c.egress_ms > 0 ? 2 : 1) : 0);
    const double comp = c.compute_ms + c.halo_exposed_ms;
    c.step_ms = std::max(comp, io);
    c.bound = comp >= io ? (c.halo_exposed_ms > 0.25 * comp ? "halo" : "compute")
              : c.egress_ms > 0 ? (c.egress_ms >= c.ingress_ms ? "egress" : "ingress")
                                : "ingress";
  }
  c.images_per_s = c.step_ms > 0 ? c.images / c.step_ms * 1e3 : 0;
  return c;
}

int pick_row_ways(Workload wl, int np, int batch, InputSource src, Decomp mode, const CostParams& p,
                  const BlockSpec& b1, const BlockSpec& b2, int H, int W) {
  if (np <= 1 || wl == Workload::DP) return 1;
  int best = 1;
  double best_ms = 1e300;
  for (int r = 1; r <= np; ++r) {
    if (np % r) continue;
    const int global = batch;
    // fewer images than row groups leaves ranks idle: still a valid candidate, the model prices it
    HybridPlan hp;
    if (!make_hybrid_plan(H, W, np, global, r, mode, hp, b1, b2)) continue;
    const double ms = model_step(wl, np, batch, r, src, mode, p, b1, b2, H, W).step_ms;
    if (ms < best_ms * (1 - 1e-9)) best_ms = ms, best = r;
  }
  return best;
}

std::string model_curve_json(Workload wl, const std::vector<int>& nps, int batch, int row_ways, InputSource src,
                             Decomp mode, const CostParams& p) {
  std::vector<StepCost> cs;
  for (int n : nps) cs.push_back(model_step(wl, n, batch, row_ways, src, mode, p));
  auto arr = [&](auto f, const char* fmt) {
    std::string s = "[";
    char b[64];
    for (size_t i = 0; i < cs.size(); ++i) {
      std::snprintf(b, sizeof b, fmt, f(cs[i]));
      s += (i ? ", " : "") + std::string(b);
    }
    return s + "]";
  };
  const double t1 = cs.empty() ? 0 : cs[0].step_ms, x1 = cs.empty() ? 0 : cs[0].images_per_s;
  const bool weak = wl == Workload::DP;
  std::string s = "{\"workload\": \"" + std::string(wl_name(wl)) + "\", \"measured\": false, \"scaling\": \"" +
                  (weak ? "weak" : "strong") + "\", ";
  s += "\"N\": " + arr([](const StepCost& c) { return c.np; }, "%d") + ", ";
  s += "\"row_ways\": " + arr([](const StepCost& c) { return c.row_ways; }, "%d") + ", ";
  s += "\"root_batch\": " + arr([](const StepCost& c) { return c.root_batch; }, "%d") + ", ";
  s += "\"step_ms\": " + arr([](const StepCost& c) { return c.step_ms; }, "%.4f") + ", ";
  s += "\"images_per_s\": " + arr([](const StepCost& c) { return c.images_per_s; }, "%.0f") + ", ";
  s += "\"speedup\": " +
       arr([&](const StepCost& c) { return weak ? c.images_per_s / x1 : t1 / c.step_ms; }, "%.3f") + ", ";
  s += "\"efficiency\": " +
       arr([&](const StepCost& c) { return (weak ? c.images_per_s / x1 : t1 / c.step_ms) / c.np; }, "%.3f") + ", ";
  s += "\"bound\": [";
  for (size_t i = 0; i < cs.size(); ++i) s += (i ? ", \"" : "\"") + cs[i].bound + "\"";
  s += "], \"steps\": [";
  for (size_t i = 0; i < cs.size(); ++i) s += (i ? ", " : "") + cs[i].json();
  std::string rate = "\"rate\": [";
  for (size_t i = 0; i < p.rate_images.size() && i < p.rate_img_s.size(); ++i)
    rate += (i ? ", [" : "[") + std::to_string(p.rate_images[i]) + ", " + std::to_string(static_cast<long>(p.rate_img_s[i])) + "]";
  rate += "], ";
  char b[1024];
  std::snprintf(b, sizeof b,
                "], \"params\": {%s\"xgmi_gbps\": %g, \"h2d_gbps\": %g, \"d2h_gbps\": %g, \"host_gbps\": %g, "
                "\"ingest_slowdown\": %g, \"dp_root_shed\": %d, \"stage1_share\": %g, \"split_penalty\": %g, \"phase_latency_ms\": %g, "
                "\"v4_fill\": %g, \"v5_chunks\": %d}}",
                rate.c_str(), p.xgmi_gbps, p.h2d_gbps, p.d2h_gbps, p.host_gbps, p.ingest_slowdown, p.dp_root_shed, p.stage1_share, p.split_penalty,
                p.phase_latency_ms, p.v4_fill, p.v5_chunks);
  return s + b;
}

}  // namespace anx
