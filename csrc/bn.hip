// BatchNorm (train + eval), activation and residual kernels for NHWC bf16.
//
// The forward conv epilogue (igemm.hip) already accumulates per-(ghost-group,
// channel) sum / sum-of-squares, so BN forward here is a single streaming pass:
//   out = act( y*scale + shift  [+ residual | + y2*scale2 + shift2] )
// with scale/shift derived on the fly from the sums (train) or running stats
// (eval).  Ghost groups reproduce the reference's scoring semantics exactly: the
// reference scores 10 separate batches of 32 in train mode (`pytorch_collab.py:95-103`),
// each normalised with its own batch statistics; here the 320-sample pool is one
// launch whose rows are split into 10 stat groups.
//
// Backward (train batch, one group) is two passes:
//   reduce: sum(dz), sum(dz*xhat) [and sum(dz*xhat2) for a BN'd shortcut sharing dz]
//   apply : dy = gamma*rstd*(dz - mean(dz) - xhat*mean(dz*xhat)); writes dgamma/dbeta
// where dz = dout * act'(out) is recomputed from the saved block output.
//
// Thread mapping: every thread keeps ONE 8-channel chunk for its whole grid-stride
// loop (the stride is a multiple of C/8), so per-channel constants are computed
// once per thread and loads/stores are 16 bytes.
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

MA_DEV void scale_shift(const float* stats, int ld, int g, int c, float inv_cnt, float eps,
                        const float* gamma, const float* beta, const float* rm, const float* rv,
                        int use_running, float& sc, float& sh) {
  float mean, var;
  if (use_running) {
    mean = rm[c];
    var = rv[c];
  } else {
    const float s = stats[(size_t)g * 2 * ld + c], ss = stats[(size_t)g * 2 * ld + ld + c];
    mean = s * inv_cnt;
    var = fmaxf(ss * inv_cnt - mean * mean, 0.f);
  }
  const float rstd = rsqrtf(var + eps);
  sc = (gamma ? gamma[c] : 1.f) * rstd;
  sh = (beta ? beta[c] : 0.f) - mean * sc;
}

MA_DEV void mean_rstd(const float* stats, int ld, int c, float inv_cnt, float eps, float& mean,
                      float& rstd) {
  const float s = stats[c], ss = stats[ld + c];
  mean = s * inv_cnt;
  rstd = rsqrtf(fmaxf(ss * inv_cnt - mean * mean, 0.f) + eps);
}

MA_DEV void chunk_range(int C8, int& stride, int& start) {
  const int T = gridDim.x * NT;
  stride = T - T % C8;
  start = blockIdx.x * NT + threadIdx.x;
}

__global__ __launch_bounds__(NT) void bn_apply_kernel(BnApplyArgs a) {
  const int C8 = a.C >> 3;
  int stride, i0;
  chunk_range(C8, stride, i0);
  if (i0 >= stride) return;
  const int c8 = i0 % C8;
  const size_t total = (size_t)a.M * C8;
  float sc[8], sh[8], sc2[8], sh2[8];
  int gcur = -1;
  for (size_t i = i0; i < total; i += stride) {
    const int row = (int)(i / C8);
    const int g = row / a.group_rows;
    if (g != gcur) {
      gcur = g;
      const int cnt = min(a.group_rows, a.M - g * a.group_rows);
      const float inv = 1.f / (float)cnt;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        scale_shift(a.stats, a.C, g, c8 * 8 + k, inv, a.eps, a.gamma, a.beta, a.rmean, a.rvar,
                    a.use_running, sc[k], sh[k]);
        if (a.res_mode == 2)
          scale_shift(a.stats2, a.C, g, c8 * 8 + k, inv, a.eps, a.gamma2, a.beta2, a.rmean2,
                      a.rvar2, a.use_running, sc2[k], sh2[k]);
      }
    }
    const size_t off = i * 8;
    const bf16x8 y = *(const bf16x8*)(a.y + off);
    bf16x8 r;
    if (a.res_mode) r = *(const bf16x8*)(a.res + off);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = bf2f(y[k]) * sc[k] + sh[k];
      if (a.res_mode == 1) v += bf2f(r[k]);
      else if (a.res_mode == 2) v += bf2f(r[k]) * sc2[k] + sh2[k];
      o[k] = f2bf(act_fwd(v, a.act));
    }
    *(bf16x8*)(a.out + off) = o;
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_reduce_kernel(BnBwdArgs a) {
  __shared__ float red[3 * 2048];
  const int C8 = a.C >> 3;
  for (int i = threadIdx.x; i < 3 * a.C; i += NT) red[i] = 0.f;
  __syncthreads();
  int stride, i0;
  chunk_range(C8, stride, i0);
  const int c8 = i0 % C8;
  const float inv = 1.f / (float)a.M;
  float mean[8], rstd[8], mean2[8], rstd2[8];
  float sdz[8], sx[8], sx2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sdz[k] = sx[k] = sx2[k] = 0.f;
    const int c = c8 * 8 + k;
    mean_rstd(a.stats, a.C, c, inv, a.eps, mean[k], rstd[k]);
    if (a.y2) mean_rstd(a.stats2, a.C, c, inv, a.eps, mean2[k], rstd2[k]);
  }
  if (i0 < stride) {
    const size_t total = (size_t)a.M * C8;
    for (size_t i = i0; i < total; i += stride) {
      const size_t off = i * 8;
      const bf16x8 d = *(const bf16x8*)(a.dout + off);
      const bf16x8 o = *(const bf16x8*)(a.out + off);
      const bf16x8 y = *(const bf16x8*)(a.y + off);
      bf16x8 y2;
      if (a.y2) y2 = *(const bf16x8*)(a.y2 + off);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float dz = bf2f(d[k]) * act_mask(bf2f(o[k]), a.act);
        sdz[k] += dz;
        sx[k] += dz * (bf2f(y[k]) - mean[k]) * rstd[k];
        if (a.y2) sx2[k] += dz * (bf2f(y2[k]) - mean2[k]) * rstd2[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c8 * 8 + k;
      atomicAdd(&red[c], sdz[k]);
      atomicAdd(&red[a.C + c], sx[k]);
      if (a.y2) atomicAdd(&red[2 * a.C + c], sx2[k]);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < a.C; c += NT) {
    atomicAdd(&a.sums[c], red[c]);
    atomicAdd(&a.sums[a.C + c], red[a.C + c]);
    if (a.y2) atomicAdd(&a.sums[2 * a.C + c], red[2 * a.C + c]);
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BnBwdArgs a) {
  const int C8 = a.C >> 3;
  const float inv = 1.f / (float)a.M;
  if (blockIdx.x == 0) {  // parameter gradients
    for (int c = threadIdx.x; c < a.C; c += NT) {
      if (a.dgamma) a.dgamma[c] = a.sums[a.C + c];
      if (a.dbeta) a.dbeta[c] = a.sums[c];
      if (a.y2) {
        if (a.dgamma2) a.dgamma2[c] = a.sums[2 * a.C + c];
        if (a.dbeta2) a.dbeta2[c] = a.sums[c];
      }
    }
  }
  int stride, i0;
  chunk_range(C8, stride, i0);
  if (i0 >= stride) return;
  const int c8 = i0 % C8;
  float k1[8], k2[8], mean[8], rstd[8], q1[8], q2[8], mean2[8], rstd2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c8 * 8 + k;
    mean_rstd(a.stats, a.C, c, inv, a.eps, mean[k], rstd[k]);
    const float gm = a.gamma ? a.gamma[c] : 1.f;
    k1[k] = gm * rstd[k];                  // gamma*rstd
    k2[k] = a.sums[c] * inv;               // mean(dz)
    q1[k] = a.sums[a.C + c] * inv;         // mean(dz*xhat)
    if (a.y2) {
      mean_rstd(a.stats2, a.C, c, inv, a.eps, mean2[k], rstd2[k]);
      q2[k] = a.sums[2 * a.C + c] * inv;
    }
  }
  const size_t total = (size_t)a.M * C8;
  for (size_t i = i0; i < total; i += stride) {
    const size_t off = i * 8;
    const bf16x8 d = *(const bf16x8*)(a.dout + off);
    const bf16x8 o = *(const bf16x8*)(a.out + off);
    const bf16x8 y = *(const bf16x8*)(a.y + off);
    bf16x8 y2, dy, dy2, dzo;
    if (a.y2) y2 = *(const bf16x8*)(a.y2 + off);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float dz = bf2f(d[k]) * act_mask(bf2f(o[k]), a.act);
      const float xh = (bf2f(y[k]) - mean[k]) * rstd[k];
      dy[k] = f2bf(k1[k] * (dz - k2[k] - xh * q1[k]));
      if (a.y2) {
        const int c = c8 * 8 + k;
        const float g2 = a.gamma2 ? a.gamma2[c] : 1.f;
        const float xh2 = (bf2f(y2[k]) - mean2[k]) * rstd2[k];
        dy2[k] = f2bf(g2 * rstd2[k] * (dz - k2[k] - xh2 * q2[k]));
      }
      dzo[k] = f2bf(dz);
    }
    *(bf16x8*)(a.dy + off) = dy;
    if (a.y2) *(bf16x8*)(a.dy2 + off) = dy2;
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
    for (int g = 0; g < ng; ++g) {
      const float s = st[(size_t)g * 2 * e.C + c], ss = st[(size_t)g * 2 * e.C + e.C + c];
      const float mean = s / cnt;
      const float var = fmaxf(ss / cnt - mean * mean, 0.f) * (cnt / fmaxf(cnt - 1.f, 1.f));
      rm = (1.f - momentum) * rm + momentum * mean;
      rv = (1.f - momentum) * rv + momentum * var;
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

void bn_apply_launch(const BnApplyArgs& a, hipStream_t st) {
  const size_t chunks = (size_t)a.M * (a.C / 8);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(chunks, a.C / 8, 4, 2048)), dim3(NT), 0, st, a);
}

void bn_bwd_launch(const BnBwdArgs& a, hipStream_t st) {
  const size_t chunks = (size_t)a.M * (a.C / 8);
  hipMemsetAsync(a.sums, 0, sizeof(float) * 3 * a.C, st);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(grid_for(chunks, a.C / 8, 16, 128)), dim3(NT), 0,
                     st, a);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(chunks, a.C / 8, 4, 2048)), dim3(NT), 0,
                     st, a);
}

void bn_running_launch(const BnRunEntry* tab, int nlayers, int maxC, float momentum,
                       hipStream_t st) {
  hipLaunchKernelGGL(bn_running_kernel, dim3((maxC + NT - 1) / NT, nlayers), dim3(NT), 0, st, tab,
                     nlayers, momentum);
}
