// K3: batched fault-domain posteriors and labelled sufficient statistics on matrix cores.
//
// Every attribution model (REF-exact naive Bayes, learned Bayes, covariance LDA; see
// models/bayes.py) is a linear-logit model: logits[b, d] = X[b, :] @ W[:, d] + bias[d],
// X = binary evidence (value >= elevated threshold, REF bayesian.go:194-243) or centred
// log1p features. One wave computes a 16-incident x 16-domain logit tile with four
// v_mfma_f64_16x16x4_f64 (K = 16 signal slots) -- float64 like REF's math.Log sums, so
// the GPU posteriors match the CPU oracle to ~1e-15 -- then does the log-sum-exp,
// argmax (ties -> lowest domain index == REF's stable sort), evidence bitmask
// (elevated & P(elevated|d) >= 0.5) and the confusion-matrix update in registers.
//
// k_stats is the "MFMA covariance step": U^T V with U = [E | X], V = [Y | X] over a batch
// of labelled incidents (K = incidents), giving E^T Y (likelihood counts), X^T Y (class
// sums) and X^T X (scatter) in one 32x32 f64 product, reduced across waves with f64
// atomics. These are the sufficient statistics the learned models are refit from.
//
// 2-fault models (models/bayes.py with_pairs) add up to kMaxPairs hypothesis columns -- every
// pair of fault domains, a noisy-OR of its members -- as up to three more 16-column MFMA tiles
// of the same K = 16 product. The log-sum-exp then runs over singles and pairs together, and
// each domain lane sums its marginal P(d in incident) = P({d}) + sum_h P(pair h holds d) with
// one 16-lane shuffle per pair; argmax / confidence are taken over the marginals.
//
// f64 MFMA C/D layout on gfx950: col = lane & 15, row = (lane >> 4) + 4 * reg
// (cdna_hip_programming.md section 3 -- NOT the f32 row map).
#include "mislo_common.h"
#include "mislo_launch.h"

namespace mislo {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// element `j` (wave-uniform, not a compile-time constant) of an accumulator, as selects
__device__ __forceinline__ double pick(const f64x4& v, int j) {
  return j == 0 ? v[0] : (j == 1 ? v[1] : (j == 2 ? v[2] : v[3]));
}

__device__ __forceinline__ double feature_x(float v, int s, const PosteriorModel& pm) {
  if (pm.mode == 0) {
    const bool e = (v == v) && v >= pm.thr[s] && ((pm.table_mask >> s) & 1u);
    return e ? 1.0 : 0.0;
  }
  const double vv = (v == v) ? (double)v : pm.nominal[s];
  return log1p(vv > 0.0 ? vv : 0.0) - pm.mean[s];
}

__device__ __forceinline__ uint32_t elevated_bits(const float* __restrict__ row, const PosteriorModel& pm) {
  uint32_t b = 0;
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    const float v = row[s];
    if ((v == v) && v >= pm.thr[s]) b |= 1u << s;
  }
  return b & pm.table_mask;
}

struct PosteriorArgs {
  const float* feat;
  const int* ng_ptr;
  int cap;
  const PosteriorModel* pm;
  const int32_t* labels;
  double *post, *conf;
  int32_t* pred;
  uint32_t *evbits, *confusion;
  const AppModel* app;      // optional application evidence (mislo_launch.h)
  const uint32_t* app_cnt;  // [G][2] the groups' application retrieval counts
};

// Application evidence of row r: -1 absent (no span of the group reported a retrieval time), 0
// present, 1 elevated. The residual is computed in double from the exact group sum and the float
// features, in the order models/bayes.py AppEvidence.residual uses, so host and device agree
// bit for bit.
__device__ __forceinline__ int app_state(const uint32_t* __restrict__ cnt, const float* __restrict__ feat, int r,
                                         double thr_ms) {
  const uint32_t n = cnt[2 * r];
  if (n == 0) return -1;
  const double mean = (double)cnt[2 * r + 1] / kAppUnitsPerMs / (double)n;
  const float* f = feat + (size_t)r * kSlots;
  double kern = 0.0;  // REF DecomposeRetrieval: dns + connect + tls
  if (f[0] == f[0]) kern += (double)f[0];
  if (f[3] == f[3]) kern += (double)f[3];
  if (f[5] == f[5]) kern += (double)f[5];
  return (mean - kern) >= thr_ms ? 1 : 0;
}
struct StatsArgs {
  const float* feat;
  const int* ng_ptr;
  int cap;
  const PosteriorModel* pm;
  const int32_t* labels;
  const float* weights;
  double *out, *count;
};

// WPG waves per 16-row group: each computes the group's logit tile (four MFMAs, cheap to repeat)
// and then the softmax / marginal / argmax of 4 / WPG of its accumulator rows. The normalisation
// is a chain of f64 exp / shuffles per row quad: with one wave per group a window's 64
// incidents ran as 4 waves of 4 serial quads (~30 us); 4 waves per group cut the chain to one.
template <int NT, int WPG = 1>
__device__ __forceinline__ void posterior_body(int blk, const PosteriorArgs& a_) {
  const float* __restrict__ feat = a_.feat;
  const int32_t* __restrict__ labels = a_.labels;
  double* __restrict__ post = a_.post;
  int32_t* __restrict__ pred = a_.pred;
  double* __restrict__ conf = a_.conf;
  uint32_t* __restrict__ evbits = a_.evbits;
  uint32_t* __restrict__ confusion = a_.confusion;
  // The model (~9 KB) is copied into LDS once, with every load in flight together: read from
  // global memory, its fields were dependent round trips to a cold L2 (a window's join evicts
  // it), several per row group since the result stores may alias the model (49 us per dispatch
  // with the 2-fault columns, most of it waiting)
  __shared__ alignas(16) PosteriorModel s_pm;
  {
    constexpr int n16 = (int)(sizeof(PosteriorModel) / 16), tail = (int)(sizeof(PosteriorModel) % 16);
    const uint4* src = reinterpret_cast<const uint4*>(a_.pm);
    uint4* dst = reinterpret_cast<uint4*>(&s_pm);
    for (int q = threadIdx.x; q < n16; q += NT) dst[q] = src[q];
    if (tail && threadIdx.x < tail)
      reinterpret_cast<uint8_t*>(&s_pm)[16 * n16 + threadIdx.x] =
          reinterpret_cast<const uint8_t*>(a_.pm)[16 * n16 + threadIdx.x];
  }
  __syncthreads();
  const PosteriorModel& pm = s_pm;
  const int G = min(*a_.ng_ptr, a_.cap);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  static_assert(WPG == 1 || WPG == 2 || WPG == 4, "waves per row group divide the 4 accumulator rows");
  constexpr int kRegs = 4 / WPG;
  const int row0 = (blk * (NT / 64 / WPG) + wave / WPG) * 16;
  const int reg0 = (wave % WPG) * kRegs;
  const int i = lane & 15;
  const int kq = lane >> 4;
  const int n_pairs = pm.n_pairs;
  // the pairs holding this lane's domain, as a bitmask
  static_assert(kMaxPairs <= 64, "pair masks are 64-bit");
  unsigned long long pmask = 0ull;
  for (int h = 0; h < n_pairs; ++h)
    if (pm.pair_a[h] == i || pm.pair_b[h] == i) pmask |= 1ull << h;
  if (row0 >= G) return;  // whole wave exits together
  // the application channel's terms of this lane's domain (and pair columns)
  const bool app_on = a_.app != nullptr && a_.app_cnt != nullptr && a_.app->on != 0;
  double app_w = 0.0, app_b = 0.0, app_thr = 0.0;
  double app_w2[3] = {0.0, 0.0, 0.0}, app_b2[3] = {0.0, 0.0, 0.0};
  uint32_t app_ev = 0u;
  if (app_on) {
    app_w = a_.app->w[i];
    app_b = a_.app->b[i];
    app_thr = a_.app->thr_ms;
    app_ev = (a_.app->dom_mask >> i) & 1u;
#pragma unroll
    for (int t = 0; t < 3; ++t)
      if (16 * t + i < kMaxPairs) {
        app_w2[t] = a_.app->w2[16 * t + i];
        app_b2[t] = a_.app->b2[16 * t + i];
      }
  }

  const int n_pt = (n_pairs + 15) >> 4;  // pair tiles (uniform over the wave)
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  f64x4 acc2[3] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int s = 4 * kk + kq;
    const int r = row0 + i;
    const double a = r < G ? feature_x(feat[(size_t)r * kSlots + s], s, pm) : 0.0;
    const double b = pm.w[s][i];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 3; ++t)
      if (t < n_pt) acc2[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, pm.w2[s][16 * t + i], acc2[t], 0, 0, 0);
  }

  const double bias = pm.bias[i];
  if (n_pt > 0) {
    double b2[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) b2[t] = (16 * t + i < n_pairs) ? pm.bias2[16 * t + i] : -INFINITY;
#pragma unroll
    for (int rr = 0; rr < kRegs; ++rr) {
      const int reg = reg0 + rr;
      const int r = row0 + kq + 4 * reg;
      const int as = (app_on && r < G) ? app_state(a_.app_cnt, feat, r, app_thr) : -1;
      double lg = pick(acc, reg) + bias;
      if (as >= 0 && lg != -INFINITY) lg += app_b + (as ? app_w : 0.0);
      double l2[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        l2[t] = (t < n_pt) ? pick(acc2[t], reg) + b2[t] : -INFINITY;
        if (as >= 0 && l2[t] != -INFINITY) l2[t] += app_b2[t] + (as ? app_w2[t] : 0.0);
      }
      double m = fmax(lg, fmax(l2[0], fmax(l2[1], l2[2])));
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) m = fmax(m, __shfl_xor(m, off, 16));
      // normalised by one reciprocal: each hypothesis' exp is taken once (not again against logz)
      const double e1 = (lg == -INFINITY) ? 0.0 : exp(lg - m);
      double e2[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) e2[t] = (l2[t] == -INFINITY) ? 0.0 : exp(l2[t] - m);
      double sum = e1 + e2[0] + e2[1] + e2[2];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 16);
      const double inv = 1.0 / sum;
      double pp[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) pp[t] = e2[t] * inv;
      double marg = e1 * inv;
      for (int h = 0; h < n_pairs; ++h) {  // pair h lives in tile h >> 4, lane h & 15
        const int t = h >> 4;
        const double v = t == 0 ? pp[0] : (t == 1 ? pp[1] : pp[2]);
        const double ph = __shfl(v, h & 15, 16);
        if ((pmask >> h) & 1ull) marg += ph;
      }
      double mm = marg;
      int am = i;
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        const double om = __shfl_xor(mm, off, 16);
        const int oa = __shfl_xor(am, off, 16);
        if (om > mm || (om == mm && oa < am)) { mm = om; am = oa; }
      }
      if (r < G) {
        post[(size_t)r * kMaxDomains + i] = marg;
        const uint32_t eb = elevated_bits(feat + (size_t)r * kSlots, pm);
        evbits[(size_t)r * kMaxDomains + i] = (eb & pm.dom_mask[i]) | ((as == 1 ? app_ev : 0u) << kAppBit);
        if (i == 0) {
          pred[r] = am;
          conf[r] = mm;
          if (labels != nullptr) {
            const int y = labels[r];
            if (y >= 0 && (y & 0xFF) < kMaxDomains) atomicAdd(confusion + (y & 0xFF) * kMaxDomains + am, 1u);
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int rr = 0; rr < kRegs; ++rr) {
    const int reg = reg0 + rr;
    const int r = row0 + kq + 4 * reg;
    const int as = (app_on && r < G) ? app_state(a_.app_cnt, feat, r, app_thr) : -1;
    double lg = pick(acc, reg) + bias;  // -inf for inactive domains
    if (as >= 0 && lg != -INFINITY) lg += app_b + (as ? app_w : 0.0);
    // max + argmax over the 16 domain lanes (ties -> lowest index)
    double m = lg;
    int am = i;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const double om = __shfl_xor(m, off, 16);
      const int oa = __shfl_xor(am, off, 16);
      if (om > m || (om == m && oa < am)) { m = om; am = oa; }
    }
    const double ex = (lg == -INFINITY) ? 0.0 : exp(lg - m);
    double sum = ex;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 16);
    const double inv = 1.0 / sum;  // the argmax's own term is exp(0) = 1: its posterior is inv
    const double p = ex * inv;
    if (r < G) {
      post[(size_t)r * kMaxDomains + i] = p;
      const uint32_t eb = elevated_bits(feat + (size_t)r * kSlots, pm);
      evbits[(size_t)r * kMaxDomains + i] = (eb & pm.dom_mask[i]) | ((as == 1 ? app_ev : 0u) << kAppBit);
      if (i == 0) {
        pred[r] = am;
        conf[r] = inv;
        if (labels != nullptr) {
          const int y = labels[r];  // primary domain in bits 0-7 (label_code: a domain set above)
          if (y >= 0 && (y & 0xFF) < kMaxDomains) atomicAdd(confusion + (y & 0xFF) * kMaxDomains + am, 1u);
        }
      }
    }
  }
}

template <int NT, int WPG>
__global__ __launch_bounds__(NT) void k_posterior(PosteriorArgs a) {
  posterior_body<NT, WPG>(blockIdx.x, a);
}

// U^T V over labelled incidents; out[32][32] f64, count[16] f64.
template <int NT, int ROWS_PER_WAVE>
__device__ __forceinline__ void stats_body(int blk, const StatsArgs& a_) {
  const float* __restrict__ feat = a_.feat;
  const int32_t* __restrict__ labels = a_.labels;
  const float* __restrict__ weights = a_.weights;
  double* __restrict__ out = a_.out;
  double* __restrict__ count = a_.count;
  const int G = min(*a_.ng_ptr, a_.cap);
  const PosteriorModel& pm = *a_.pm;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int base = (blk * (NT / 64) + wave) * ROWS_PER_WAVE;
  if (base >= G) return;
  const int i = lane & 15;
  const int kq = lane >> 4;
  f64x4 t00 = {0, 0, 0, 0}, t01 = {0, 0, 0, 0}, t10 = {0, 0, 0, 0}, t11 = {0, 0, 0, 0};
  for (int r0 = base; r0 < base + ROWS_PER_WAVE && r0 < G; r0 += 4) {
    const int r = r0 + kq;
    double e = 0.0, x = 0.0, y = 0.0;
    if (r < G) {
      const int lab = labels[r];
      const double wgt = weights ? (double)weights[r] : 1.0;
      if (lab >= 0) {
        const float v = feat[(size_t)r * kSlots + i];
        e = ((v == v) && v >= pm.thr[i]) ? 1.0 : 0.0;
        const double vv = (v == v) ? (double)v : pm.nominal[i];
        x = log1p(vv > 0.0 ? vv : 0.0);
        // label_code: bits 0-7 the primary domain, bits 8-23 the incident's domain set (a
        // multi-fault incident): a soft label spread evenly over the set
        const uint32_t set = ((uint32_t)lab >> 8) & 0xFFFFu;
        y = set ? (((set >> i) & 1u) ? wgt / (double)__popc(set) : 0.0) : ((lab & 0xFF) == i ? wgt : 0.0);
        if (y != 0.0) atomicAdd(count + i, y);
      }
    }
    // A = U^T (rows = U columns, k = incident), B = V (k = incident, cols = V columns)
    t00 = __builtin_amdgcn_mfma_f64_16x16x4f64(e, y, t00, 0, 0, 0);  // E^T Y
    t01 = __builtin_amdgcn_mfma_f64_16x16x4f64(e, x, t01, 0, 0, 0);  // E^T X
    t10 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, t10, 0, 0, 0);  // X^T Y
    t11 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, t11, 0, 0, 0);  // X^T X
  }
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int rr = kq + 4 * reg;
    atomicAdd(out + (size_t)rr * 32 + i, t00[reg]);
    atomicAdd(out + (size_t)rr * 32 + 16 + i, t01[reg]);
    atomicAdd(out + (size_t)(16 + rr) * 32 + i, t10[reg]);
    atomicAdd(out + (size_t)(16 + rr) * 32 + 16 + i, t11[reg]);
  }
}

template <int NT, int ROWS_PER_WAVE>
__global__ __launch_bounds__(NT) void k_stats(StatsArgs a) {
  stats_body<NT, ROWS_PER_WAVE>(blockIdx.x, a);
}

// Posterior + sufficient statistics of a learning window in ONE launch: the two read the same
// features and model and write disjoint outputs, and each is a single latency-bound
// workgroup at the default 64 incidents; back to back they cost two serial launches.
template <int NT, int ROWS_PER_WAVE>
__global__ __launch_bounds__(NT) void k_posterior_stats(PosteriorArgs p, StatsArgs st, int n_post_blocks) {
  if ((int)blockIdx.x < n_post_blocks) posterior_body<NT>(blockIdx.x, p);
  else stats_body<NT, ROWS_PER_WAVE>(blockIdx.x - n_post_blocks, st);
}

// On-device refit of the learned naive Bayes (models/bayes.py NaiveBayes.learned) from
// the accumulated, all-reduced sufficient statistics: posterior-mean likelihoods
//   p_sd = max((c_sd + alpha * p0_sd) / (n_d + alpha), floor_sd),  pi_d = (n_d + pp) / (N + pp * D)
// turned into the linear-logit model in place (w, bias, evidence masks). Runs on the
// compute stream between windows, so online learning needs no host round trip.
// stats: [32 x 32] f64 (rows 0-15 = E^T Y) followed by count[16]; p0: [16 x 16] f64, the Beta
// prior's table (REF's expert table or the random-init one); floor (optional): [16 x 16] f64
// minimum likelihoods (REF's "unknown" column: chance elevations, models/bayes.py unknown_floor).
// add (optional, same layout): a window's all-reduced statistics, folded into stats first
// (one launch instead of an elementwise add plus the refit on the compute stream).
// inv_temp scales every logit (w and bias; the calibration temperature T = 1 / inv_temp fitted on
// held-out windows, models/train.py): argmax and evidence are unchanged, the posteriors are
// flatter for T > 1 (REF's coverage metric counts hypotheses >= 0.10). A domain with less than
// min_count labelled mass is inactive (bias -inf). cap_dom (>= 0): that domain's prior is capped
// at the largest prior of the other active domains (the no-fault class must not win on its
// label frequency alone).
__global__ __launch_bounds__(256) void k_refit_nb(double* __restrict__ stats, const double* __restrict__ add,
                                                  const double* __restrict__ p0, const double* __restrict__ floor_tab,
                                                  double alpha, double prior_pseudo, int n_dom, double inv_temp,
                                                  double min_count, int cap_dom, double ceil,
                                                  PosteriorModel* __restrict__ pm) {
  __shared__ double s_logpn[kSlots][kMaxDomains];
  __shared__ double s_pe[kSlots][kMaxDomains];
  __shared__ double s_logpi[kMaxDomains];
  __shared__ double s_pnorm;
  __shared__ uint32_t s_mask[kMaxDomains];
  const double* count = stats + 32 * 32;
  const int t = threadIdx.x;
  if (add)
    for (int i = t; i < 32 * 32 + kMaxDomains; i += 256) stats[i] += add[i];
  if (t < kMaxDomains) s_mask[t] = 0u;
  __syncthreads();
  {
    const int sl = t >> 4, d = t & 15;  // 256 threads = 16 slots x 16 domain columns
    if (d < n_dom) {
      const double n = count[d];
      const double c = stats[sl * 32 + d];
      double p = (c + alpha * p0[sl * 16 + d]) / (n + alpha);
      if (floor_tab) p = fmax(p, floor_tab[sl * 16 + d]);
      p = fmin(p, ceil);  // the learned likelihood cap (models/bayes.py NaiveBayes.learned ceil)
      const double pe = fmin(fmax(p, 0.01), 0.99), pn = fmin(fmax(1.0 - p, 0.01), 0.99);
      pm->w[sl][d] = (log(pe) - log(pn)) * inv_temp;
      s_logpn[sl][d] = log(pn);
      s_pe[sl][d] = pe;
      if (p >= 0.5) atomicOr(&s_mask[d], 1u << sl);
    } else {
      pm->w[sl][d] = 0.0;
      s_logpn[sl][d] = 0.0;
      s_pe[sl][d] = 0.0;
    }
  }
  if (t < kMaxDomains) {
    if (t < n_dom && count[t] >= min_count) {
      double N = 0.0;
      for (int d = 0; d < n_dom; ++d) N += count[d];
      s_logpi[t] = log((count[t] + prior_pseudo) / (N + prior_pseudo * (double)n_dom));
    } else {
      s_logpi[t] = -__builtin_inf();
    }
  }
  __syncthreads();
  double logpi_t = t < kMaxDomains ? s_logpi[t] : 0.0;
  if (t == cap_dom && logpi_t > -__builtin_inf()) {
    double mx = -__builtin_inf();
    for (int d = 0; d < n_dom; ++d)
      if (d != t) mx = fmax(mx, s_logpi[d]);
    if (mx > -__builtin_inf()) logpi_t = fmin(logpi_t, mx);
  }
  __syncthreads();  // every read of s_logpi above is done before the capped prior is stored
  if (t < kMaxDomains) {
    if (logpi_t > -__builtin_inf()) {
      double b = logpi_t;
      for (int sl = 0; sl < kSlots; ++sl) b += s_logpn[sl][t];
      if (pm->n_pairs > 0) b += log1p(-pm->pair_rho);  // singles keep 1 - rho of the prior
      pm->bias[t] = b * inv_temp;
      pm->dom_mask[t] = s_mask[t];
    } else {
      pm->bias[t] = -__builtin_inf();
      pm->dom_mask[t] = 0u;
    }
    s_logpi[t] = logpi_t;
  }
  if (t == 0) {
    pm->table_mask = 0xFFFFu;
    pm->mode = 0;
  }
  const int n_pairs = pm->n_pairs;
  const double rho = pm->pair_rho;
  if (n_pairs <= 0) return;
  // 2-fault columns (models/bayes.py with_pairs): noisy-OR likelihoods q = 1 - (1-p_a)(1-p_b),
  // prior rho * pi_a pi_b / sum over the active pairs
  __syncthreads();
  if (t == 0) {
    double z = 0.0;
    for (int h = 0; h < n_pairs; ++h) {
      const double pr = s_logpi[pm->pair_a[h]] + s_logpi[pm->pair_b[h]];
      if (pr > -__builtin_inf()) z += exp(pr);
    }
    s_pnorm = log(z);
  }
  __syncthreads();
  for (int h = t; h < n_pairs; h += 256) {
    const int a = pm->pair_a[h], b = pm->pair_b[h];
    const double pr = s_logpi[a] + s_logpi[b];
    if (!(pr > -__builtin_inf())) {
      for (int sl = 0; sl < kSlots; ++sl) pm->w2[sl][h] = 0.0;
      pm->bias2[h] = -__builtin_inf();
      continue;
    }
    double bb = log(rho) + pr - s_pnorm;
    for (int sl = 0; sl < kSlots; ++sl) {
      const double q0 = 1.0 - (1.0 - s_pe[sl][a]) * (1.0 - s_pe[sl][b]);
      const double q = fmin(fmax(q0, 0.01), 0.99), qn = fmin(fmax(1.0 - q, 0.01), 0.99);
      pm->w2[sl][h] = (log(q) - log(qn)) * inv_temp;
      bb += log(qn);
    }
    pm->bias2[h] = bb * inv_temp;
  }
}

void launch_refit_nb(double* stats, const double* add, const double* p0, double alpha, double prior_pseudo, int n_dom,
                     PosteriorModel* pm, hipStream_t stream, double inv_temp, double min_count, const double* floor_tab,
                     int cap_dom, double ceil) {
  hipLaunchKernelGGL(k_refit_nb, dim3(1), dim3(256), 0, stream, stats, add, p0, floor_tab, alpha, prior_pseudo, n_dom,
                     inv_temp, min_count, cap_dom, ceil, pm);
}

constexpr int kPostNT = 256, kStatsRPW = 256;
static int posterior_grid(int cap) {
  const int rows_per_block = (kPostNT / 64) * 16;
  const int g = (cap + rows_per_block - 1) / rows_per_block;
  return g > 0 ? g : 1;
}
static int stats_grid(int cap) {
  const int rows_per_block = (kPostNT / 64) * kStatsRPW;
  const int g = (cap + rows_per_block - 1) / rows_per_block;
  return g > 0 ? g : 1;
}

void launch_posterior(const float* feat, const int* ng_dev, int cap, const PosteriorModel* pm, const int32_t* labels,
                      double* post, int32_t* pred, double* conf, uint32_t* evbits, uint32_t* confusion,
                      hipStream_t stream, const AppModel* app, const uint32_t* app_cnt) {
  const PosteriorArgs a{feat, ng_dev, cap, pm, labels, post, conf, pred, evbits, confusion, app, app_cnt};
  // 16 waves per workgroup, 4 per 16-row group: a window's 64 incidents in one workgroup
  constexpr int kWPG = 4, kNT = 1024, kRowsPerBlock = kNT / 64 / kWPG * 16;
  hipLaunchKernelGGL((k_posterior<kNT, kWPG>), dim3(cap > 0 ? (cap + kRowsPerBlock - 1) / kRowsPerBlock : 1), dim3(kNT),
                     0, stream, a);
}

void launch_stats(const float* feat, const int* ng_dev, int cap, const PosteriorModel* pm, const int32_t* labels,
                  const float* weights, double* out, double* count, hipStream_t stream) {
  const StatsArgs a{feat, ng_dev, cap, pm, labels, weights, out, count};
  hipLaunchKernelGGL((k_stats<kPostNT, kStatsRPW>), dim3(stats_grid(cap)), dim3(kPostNT), 0, stream, a);
}

void launch_posterior_stats(const float* feat, const int* ng_dev, int cap, const PosteriorModel* pm,
                            const int32_t* labels, double* post, int32_t* pred, double* conf, uint32_t* evbits,
                            uint32_t* confusion, const int32_t* stat_labels, const float* weights, double* out,
                            double* count, hipStream_t stream, const AppModel* app, const uint32_t* app_cnt) {
  const PosteriorArgs p{feat, ng_dev, cap, pm, labels, post, conf, pred, evbits, confusion, app, app_cnt};
  const StatsArgs st{feat, ng_dev, cap, pm, stat_labels, weights, out, count};
  const int gp = posterior_grid(cap);
  hipLaunchKernelGGL((k_posterior_stats<kPostNT, kStatsRPW>), dim3(gp + stats_grid(cap)), dim3(kPostNT), 0, stream, p,
                     st, gp);
}

}  // namespace mislo
