// BatchNorm (train + eval), activation and residual kernels for NHWC bf16.
//
// The forward conv epilogue (igemm.hip) already accumulates per-(ghost-group,
// channel) sum / sum-of-squares, so BN forward here is a single streaming pass:
//   out = act( y*scale + shift  [+ residual | + y2*scale2 + shift2] )
// with scale/shift derived from the sums (train) or running stats (eval).  Ghost
// groups reproduce the reference's scoring semantics exactly: the reference
// scores 10 separate batches of 32 in train mode (`pytorch_collab.py:95-103`),
// each normalised with its own batch statistics; here the 320-sample pool is one
// launch whose rows are split into 10 stat groups (grid.y = group).
//
// Backward (train batch, one group) is two passes:
//   reduce: sum(dz), sum(dz*xhat) [and sum(dz*xhat2) for a BN'd shortcut sharing dz]
//   apply : dy = gamma*rstd*(dz - mean(dz) - xhat*mean(dz*xhat)); writes dgamma/dbeta
// where dz = dout * act'(out) is recomputed from the saved block output.
//
// Thread mapping: every thread owns ONE 8-channel chunk for its whole loop (the
// row stride is a multiple of C/8), so its per-channel constants are loaded once,
// as 2 x float4 per array, all issued back to back -- never as conditional scalar
// loads, which hipcc serialises behind one vmcnt(0) each (a ~15 us prologue).
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

MA_DEV float act_fwd(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}
// derivative from the activation OUTPUT
MA_DEV float act_mask(float out, int act) {
  if (act == 1) return out > 0.f ? 1.f : 0.f;
  if (act == 2) return (out > 0.f && out < 6.f) ? 1.f : 0.f;
  return 1.f;
}

MA_DEV void load8(const float* p, float (&v)[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// scale/shift for 8 channels: from batch sums (sum, sumsq) or running (mean, var).
MA_DEV void scale_shift8(const float* mean_or_sum, const float* var_or_sq, bool running,
                         float inv_cnt, float eps, const float* gamma, const float* beta,
                         float (&sc)[8], float (&sh)[8]) {
  float a[8], b[8], g[8], be[8];
  load8(mean_or_sum, a);
  load8(var_or_sq, b);
  load8(gamma, g);
  load8(beta, be);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float mean, var;
    if (running) {
      mean = a[k];
      var = b[k];
    } else {
      mean = a[k] * inv_cnt;
      var = fmaxf(b[k] * inv_cnt - mean * mean, 0.f);
    }
    sc[k] = g[k] * rsqrtf(var + eps);
    sh[k] = be[k] - mean * sc[k];
  }
}

MA_DEV void mean_rstd8(const float* stats, int ld, float inv_cnt, float eps, float (&mean)[8],
                       float (&rstd)[8]) {
  float s[8], ss[8];
  load8(stats, s);
  load8(stats + ld, ss);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = s[k] * inv_cnt;
    rstd[k] = rsqrtf(fmaxf(ss[k] * inv_cnt - mean[k] * mean[k], 0.f) + eps);
  }
}

// 16-byte store, streaming (nontemporal) when NTS: the large-batch passes write tensors far
// larger than L2 + the Infinity Cache that the next kernel re-reads from HBM anyway
template <bool NTS>
MA_DEV void st16(bf16* p, bf16x8 v) {
  if constexpr (NTS) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), (u32x4*)p);
  else *(bf16x8*)p = v;
}

// grid.x covers the rows of ONE stat group (grid.y = group), stride multiple of C/8.
// ACT / RES are compile-time (activation 0-2, residual mode 0-2): with runtime values the
// per-element code evaluated every activation and residual form and selected.
template <int ACT, int RES, bool NTS>
__global__ __launch_bounds__(NT) void bn_apply_kernel(BnApplyArgs a) {
  const int C8 = a.C >> 3;
  const int T = gridDim.x * NT;
  const int stride = T - T % C8;
  const int i0 = blockIdx.x * NT + threadIdx.x;
  if (i0 >= stride) return;
  const int c8 = i0 % C8, c = c8 * 8;
  const int g = blockIdx.y;
  const int row0 = g * a.group_rows, row1 = min(a.M, row0 + a.group_rows);
  const int rpi = stride / C8;
  // U rows per trip with every load issued before the first use (clamped rows, unconditional
  // loads); the first trip's rows are requested BEFORE the per-channel constants, so a small
  // launch pays one memory latency up front instead of two
  constexpr int U = 4;
  bf16x8 y[U], r[U];
  auto load = [&](int rb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = (size_t)min(rb + u * rpi, row1 - 1) * a.C + c;
      y[u] = *(const bf16x8*)(a.y + off);
      if (RES) r[u] = *(const bf16x8*)(a.res + off);
    }
  };
  int row = row0 + i0 / C8;
  if (row < row1) load(row);
  const float inv = 1.f / (float)(row1 - row0);
  const bool run = a.use_running != 0;
  float sc[8], sh[8], sc2[8], sh2[8];
  {
    const float* s0 = run ? a.rmean + c : a.stats + (size_t)g * 2 * a.C + c;
    const float* s1 = run ? a.rvar + c : s0 + a.C;
    scale_shift8(s0, s1, run, inv, a.eps, a.gamma + c, a.beta + c, sc, sh);
  }
  if (RES == 2) {
    const float* s0 = run ? a.rmean2 + c : a.stats2 + (size_t)g * 2 * a.C + c;
    const float* s1 = run ? a.rvar2 + c : s0 + a.C;
    scale_shift8(s0, s1, run, inv, a.eps, a.gamma2 + c, a.beta2 + c, sc2, sh2);
  }
  for (; row < row1; row += U * rpi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (row + u * rpi >= row1) break;
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = bf2f(y[u][k]) * sc[k] + sh[k];
        if (RES == 1) v += bf2f(r[u][k]);
        else if (RES == 2) v += bf2f(r[u][k]) * sc2[k] + sh2[k];
        o[k] = f2bf(act_fwd(v, ACT));
      }
      st16<NTS>(a.out + (size_t)(row + u * rpi) * a.C + c, o);
    }
    if (row + U * rpi < row1) load(row + U * rpi);
  }
}

template <int ACT, bool TWO>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_kernel(BnBwdArgs a) {
  __shared__ float red[3 * 2048];
  const int C8 = a.C >> 3;
  constexpr bool two = TWO;
  for (int i = threadIdx.x; i < 3 * a.C; i += NT) red[i] = 0.f;
  __syncthreads();
  const int T = gridDim.x * NT;
  const int stride = T - T % C8;
  const int i0 = blockIdx.x * NT + threadIdx.x;
  const int c8 = i0 % C8, c = c8 * 8;
  const float inv = 1.f / (float)a.M;
  float mean[8], rstd[8], mean2[8], rstd2[8];
  float sdz[8], sx[8], sx2[8];
  mean_rstd8(a.stats + c, a.C, inv, a.eps, mean, rstd);
  if (two) mean_rstd8(a.stats2 + c, a.C, inv, a.eps, mean2, rstd2);
#pragma unroll
  for (int k = 0; k < 8; ++k) sdz[k] = sx[k] = sx2[k] = 0.f;
  if (i0 < stride) {
    const int rpi = stride / C8;
    // 4 rows per trip: all 12-16 loads of a trip are issued before the first use, so
    // a thread exposes one memory latency per 4 rows instead of one per row
    constexpr int U = 4;
    for (int row = i0 / C8; row < a.M; row += U * rpi) {
      bf16x8 d[U], o[U], y[U], y2[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = min(row + u * rpi, a.M - 1);
        const size_t off = (size_t)r * a.C + c;
        d[u] = *(const bf16x8*)(a.dout + off);
        o[u] = *(const bf16x8*)(a.out + off);
        y[u] = *(const bf16x8*)(a.y + off);
        if (two) y2[u] = *(const bf16x8*)(a.y2 + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (row + u * rpi >= a.M) break;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dz = bf2f(d[u][k]) * act_mask(bf2f(o[u][k]), ACT);
          sdz[k] += dz;
          sx[k] += dz * (bf2f(y[u][k]) - mean[k]) * rstd[k];
          if (two) sx2[k] += dz * (bf2f(y2[u][k]) - mean2[k]) * rstd2[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(&red[c + k], sdz[k]);
      atomicAdd(&red[a.C + c + k], sx[k]);
      if (two) atomicAdd(&red[2 * a.C + c + k], sx2[k]);
    }
  }
  __syncthreads();
  float* sums = a.sums + (size_t)(blockIdx.x % SUMS_R) * 3 * a.C;   // replica (igemm.h SUMS_R)
  for (int j = threadIdx.x; j < a.C; j += NT) {
    atomicAdd(&sums[j], red[j]);
    atomicAdd(&sums[a.C + j], red[a.C + j]);
    if (two) atomicAdd(&sums[2 * a.C + j], red[2 * a.C + j]);
  }
}

// total of the SUMS_R replicas of [SUMS_R][3][C] sums at (row h, channel j)
MA_DEV float sum_sums(const float* sums, int C, int h, int j) {
  float v = 0.f;
#pragma unroll
  for (int r = 0; r < SUMS_R; ++r) v += sums[((size_t)r * 3 + h) * C + j];
  return v;
}

template <int ACT, bool TWO>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float tot[3 * 2048];   // replicas' totals [3][C]
  const int C8 = a.C >> 3;
  constexpr bool two = TWO;
  const float inv = 1.f / (float)a.M;
  // fold the SUMS_R replicas once per block (each value SUMS_R loads, shared by every thread)
  for (int j = threadIdx.x; j < (two ? 3 : 2) * a.C; j += NT)
    tot[j] = sum_sums(a.sums, a.C, j / a.C, j % a.C);
  __syncthreads();
  if (blockIdx.x == 0) {  // parameter gradients
    for (int j = threadIdx.x; j < a.C; j += NT) {
      if (a.dgamma) a.dgamma[j] = tot[a.C + j];
      if (a.dbeta) a.dbeta[j] = tot[j];
      if (two) {
        if (a.dgamma2) a.dgamma2[j] = tot[2 * a.C + j];
        if (a.dbeta2) a.dbeta2[j] = tot[j];
      }
    }
  }
  const int T = gridDim.x * NT;
  const int stride = T - T % C8;
  const int i0 = blockIdx.x * NT + threadIdx.x;
  if (i0 >= stride) return;
  const int c8 = i0 % C8, c = c8 * 8;
  const int rpi = stride / C8;
  // the next row's tensors are requested before this row's math (and the first row's before
  // the per-channel constants): one exposed memory latency per launch, not per row
  bf16x8 d, o, y, y2;
  auto load = [&](int rw) {
    const size_t off = (size_t)rw * a.C + c;
    d = *(const bf16x8*)(a.dout + off);
    o = *(const bf16x8*)(a.out + off);
    y = *(const bf16x8*)(a.y + off);
    if (two) y2 = *(const bf16x8*)(a.y2 + off);
  };
  int row = i0 / C8;
  if (row < a.M) load(row);
  float mean[8], rstd[8], gm[8], sdz[8], sx[8], mean2[8], rstd2[8], gm2[8], sx2[8];
  mean_rstd8(a.stats + c, a.C, inv, a.eps, mean, rstd);
  load8(a.gamma + c, gm);
  // (16-byte LDS reads, indexed as f32x4 so the compiler knows the alignment: eight scalar
  // reads -- or ds_read2_b32 pairs when it could not prove base % 4 == 0 -- at an 8-float lane
  // stride were 8-way bank conflicts, 5.8-13.6 conflict cycles per LDS instruction,
  // profiles/r4/pmc/final_step_pass.txt)
  auto tot8 = [&](int base, float (&v)[8]) {
    const f32x4* t4 = (const f32x4*)tot + (base >> 2);   // base = h * C + c, C % 8 == 0
    const f32x4 lo = t4[0], hi = t4[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = lo[k];
      v[4 + k] = hi[k];
    }
  };
  tot8(c, sdz);
  tot8(a.C + c, sx);
  if (two) {
    mean_rstd8(a.stats2 + c, a.C, inv, a.eps, mean2, rstd2);
    load8(a.gamma2 + c, gm2);
    tot8(2 * a.C + c, sx2);
  }
  float k1[8], k2[8], q1[8], k3[8], q2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    k1[k] = gm[k] * rstd[k];      // gamma*rstd
    k2[k] = sdz[k] * inv;         // mean(dz)
    q1[k] = sx[k] * inv;          // mean(dz*xhat)
    if (two) {
      k3[k] = gm2[k] * rstd2[k];
      q2[k] = sx2[k] * inv;
    }
  }
  for (; row < a.M; row += rpi) {
    const bf16x8 dc = d, oc = o, yc = y, y2c = y2;
    if (row + rpi < a.M) load(row + rpi);
    const size_t off = (size_t)row * a.C + c;
    bf16x8 dy, dy2, dzo;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float dz = bf2f(dc[k]) * act_mask(bf2f(oc[k]), ACT);
      const float xh = (bf2f(yc[k]) - mean[k]) * rstd[k];
      dy[k] = f2bf(k1[k] * (dz - k2[k] - xh * q1[k]));
      if (two) {
        const float xh2 = (bf2f(y2c[k]) - mean2[k]) * rstd2[k];
        dy2[k] = f2bf(k3[k] * (dz - k2[k] - xh2 * q2[k]));
      }
      dzo[k] = f2bf(dz);
    }
    *(bf16x8*)(a.dy + off) = dy;
    if (two) *(bf16x8*)(a.dy2 + off) = dy2;
    if (a.dz) *(bf16x8*)(a.dz + off) = dzo;
  }
}

// Running-statistics update for every BN layer in one launch, applying the
// momentum updates in the reference's order: the train batch first, then the
// scoring groups (`pytorch_collab.py:132` before `:159`), each with the unbiased
// variance, as nn.BatchNorm2d does.
__global__ __launch_bounds__(NT) void bn_running_kernel(const BnRunEntry* tab, int nlayers,
                                                        float momentum) {
  const BnRunEntry e = tab[blockIdx.y];
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c == 0 && e.nbt) *e.nbt += e.n_train + e.n_score;
  if (c >= e.C) return;
  float rm = e.rmean[c], rv = e.rvar[c];
  for (int pass = 0; pass < 2; ++pass) {
    const float* st = pass == 0 ? e.stats_train : e.stats_score;
    const int ng = pass == 0 ? e.n_train : e.n_score;
    const float cnt = pass == 0 ? e.cnt_train : e.cnt_score;
    // the groups' sums are loaded 8 at a time before the (sequential) momentum folds, so the
    // loads of a batch are in flight together instead of one dependent round trip per group
    for (int g0 = 0; g0 < ng; g0 += 8) {
      float s8[8], ss8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const size_t o = (size_t)(g0 + j) * 2 * e.C + c;
        s8[j] = g0 + j < ng ? st[o] : 0.f;
        ss8[j] = g0 + j < ng ? st[o + e.C] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (g0 + j >= ng) break;
        const float mean = s8[j] / cnt;
        const float var = fmaxf(ss8[j] / cnt - mean * mean, 0.f) * (cnt / fmaxf(cnt - 1.f, 1.f));
        rm = (1.f - momentum) * rm + momentum * mean;
        rv = (1.f - momentum) * rv + momentum * var;
      }
    }
  }
  e.rmean[c] = rm;
  e.rvar[c] = rv;
}

int grid_for(size_t chunks, int C8, int per_thread, int cap) {
  size_t blocks = (chunks + (size_t)NT * per_thread - 1) / ((size_t)NT * per_thread);
  if (blocks < 1) blocks = 1;
  if ((int)blocks > cap) blocks = cap;
  // at least one full period of C8 chunks must fit in the grid stride
  const size_t need = ((size_t)C8 + NT - 1) / NT;
  if (blocks < need) blocks = need;
  return (int)blocks;
}
}  // namespace

// outputs of at least this many bytes leave through streaming stores (bn_configure): the
// large-batch passes (ResNet-50 B = 1280: 0.5-2 GB) measured 1-4 % faster with them
// (bench/bn_bench.py, profiles/r6/bn_bench.jsonl); small ones stay cacheable for their reader
static long long g_bn_nt_min = 256ll << 20;

void bn_configure(long long nt_min_bytes) { g_bn_nt_min = nt_min_bytes; }

void bn_apply_launch(const BnApplyArgs& a, hipStream_t st) {
  const int G = (a.M + a.group_rows - 1) / a.group_rows;
  const size_t chunks = (size_t)a.group_rows * (a.C / 8);
  const int gx = grid_for(chunks, a.C / 8, 4, (2048 + G - 1) / G);
  const dim3 grid(gx, G);
  const bool nts = (long long)a.M * a.C * 2 >= g_bn_nt_min;
#define BN_APPLY_CASE(A, R)                                                             \
  if (a.act == A && a.res_mode == R) {                                                  \
    if (nts) hipLaunchKernelGGL((bn_apply_kernel<A, R, true>), grid, dim3(NT), 0, st, a); \
    else hipLaunchKernelGGL((bn_apply_kernel<A, R, false>), grid, dim3(NT), 0, st, a);    \
    return;                                                                             \
  }
  BN_APPLY_CASE(0, 0) BN_APPLY_CASE(0, 1) BN_APPLY_CASE(0, 2)
  BN_APPLY_CASE(1, 0) BN_APPLY_CASE(1, 1) BN_APPLY_CASE(1, 2)
  BN_APPLY_CASE(2, 0) BN_APPLY_CASE(2, 1) BN_APPLY_CASE(2, 2)
#undef BN_APPLY_CASE
  throw std::runtime_error("bn_apply: act must be 0-2 and res_mode 0-2");
}

void bn_bwd_launch(const BnBwdArgs& a, hipStream_t st) {
  // a.sums must be zero on entry (the engine zeroes one arena per step)
  const size_t chunks = (size_t)a.M * (a.C / 8);
  // 4 chunks per thread (one trip): measured at the MobileNetV2 train-batch shapes 4 / 8 / 16 /
  // 32 / 64 chunks -> 179 / 186 / 218 / 295 / 453 us over the net (a round-3 probe, since removed):
  // the loop is latency-bound, not bound by the blocks' final atomics
  // activation and shortcut-BN presence are compile-time (runtime values made the per-element
  // code evaluate every activation form and select)
  const bool two = a.y2 != nullptr;
  if (a.act < 0 || a.act > 2) throw std::runtime_error("bn_bwd: act must be 0-2");
  // both kernels fold the sums through static LDS arrays of [3][2048] floats
  if (a.C > 2048) throw std::runtime_error("bn_bwd: at most 2048 channels");
  const dim3 g1(grid_for(chunks, a.C / 8, 4, 256)), g2(grid_for(chunks, a.C / 8, 4, 2048));
#define BN_BWD_CASE(A, T)                                                                 \
  if (a.act == A && two == T) {                                                           \
    if (a.phases & 1) hipLaunchKernelGGL((bn_bwd_reduce_kernel<A, T>), g1, dim3(NT), 0, st, a); \
    if (a.phases & 2) hipLaunchKernelGGL((bn_bwd_apply_kernel<A, T>), g2, dim3(NT), 0, st, a);  \
    return;                                                                               \
  }
  BN_BWD_CASE(0, false) BN_BWD_CASE(0, true) BN_BWD_CASE(1, false) BN_BWD_CASE(1, true)
  BN_BWD_CASE(2, false) BN_BWD_CASE(2, true)
#undef BN_BWD_CASE
}

void bn_running_launch(const BnRunEntry* tab, int nlayers, int maxC, float momentum,
                       hipStream_t st) {
  hipLaunchKernelGGL(bn_running_kernel, dim3((maxC + NT - 1) / NT, nlayers), dim3(NT), 0, st, tab,
                     nlayers, momentum);
}
