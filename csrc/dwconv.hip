// Depthwise 3x3 convolution (MobileNetV2 inverted residuals), NHWC bf16, fp32 weights [C][3][3].
//
// Depthwise conv has no reduction over channels, so there is nothing for MFMA to do: it is a
// bandwidth / latency problem.  Design (per thread = one 16-byte chunk of 8 channels):
//
//   fwd   : a strip of DWL outputs along W.  The 3 x ((DWL-1)*S+3) input window is loaded once
//           as 16-byte vectors and reused by the DWL outputs (4.5 loads/output at stride 1
//           instead of 9); the thread's 72 weights are loaded once (18 x float4) into registers.
//           BN batch statistics of the bf16-rounded outputs are fused: LDS float atomics per
//           block, one global atomic per channel per block (ghost-BN groups respected).
//   dgrad : the same strip shape over the input grid (stride 1: a correlation with the flipped
//           taps through a sliding dy window; stride 2: parity-filtered gather).
//   wgrad : one thread per (image, output row, chunk) walks the row with a sliding 3x3 input
//           window (3 new loads per output at stride 1), 72 fp32 accumulators in registers, then
//           LDS reduction across the block and one global atomic per (channel, tap) per block.
//           With a slab the rows are split into column segments (shorter serial walks, a
//           larger grid) and a second kernel sums the blocks' partials: with atomics the
//           split measured slower (382 -> 568 us/step on MobileNetV2, the atomics contend).
//
// Thread index -> (chunk fastest, then strip, row, image): adjacent lanes touch adjacent 16 B
// chunks of the same pixel, so every wave access is a contiguous run of the NHWC row.
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace {
constexpr int DT = 256;
constexpr int DWL = 4;

MA_DEV void load_w72(const float* w, int c8, float (&wr)[9][8]) {
  const f32x4* src = (const f32x4*)(w + (size_t)c8 * 72);
  float t[72];
#pragma unroll
  for (int i = 0; i < 18; ++i) {
    const f32x4 v = src[i];
    t[4 * i] = v.x;
    t[4 * i + 1] = v.y;
    t[4 * i + 2] = v.z;
    t[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) wr[tap][k] = t[k * 9 + tap];
}

MA_DEV bf16x8 ld8(const bf16* p, bool ok) {
  bf16x8 v;
  if (ok) {
    v = *(const bf16x8*)p;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = f2bf(0.f);
  }
  return v;
}

constexpr int ST_LD = 17;   // floats per thread row of the forward's BN partials (odd stride)
// LOOP: one statistics group (the train batch) on a capped grid that walks the strips (the
// stride a multiple of C8, so a thread keeps its channels): fewer blocks add the BN sums, which
// contend at the memory side (profiles/r5/stats_cost/: B = 32 dw 96 ch 16.8 us with, 8.4 without)
// DH: output rows per thread.  Each loaded input row (and, with PRO, its BN transform -- most of
// the kernel's VALU) serves DH output rows: DH = 2 loads / transforms 4 rows per 2 output rows
// at stride 1 instead of 6
template <int S, bool PRO, bool LOOP, int DH>
__global__ __launch_bounds__(DT) void dw_fwd_kernel(DwArgs a) {
  extern __shared__ float part[];  // [DT][ST_LD] per-thread BN partial sums (sum, sumsq)
  const int C8 = a.C >> 3, QS = (a.Q + DWL - 1) / DWL;
  const int PR = (a.P + DH - 1) / DH;             // row groups per image
  const int per_img = PR * QS * C8;
  const int total = a.N * per_img;
  const int g0 = blockIdx.x * DT, gt = g0 + threadIdx.x;
  const int imgs_per_group = a.group_rows / (a.P * a.Q);
  const bool one_group = LOOP;
  const int T = gridDim.x * DT, stride = LOOP ? T - T % C8 : T;
  const int lim = min(total, stride);
  const int gfirst = (g0 / per_img) / imgs_per_group;
  const int glast = (min(lim - 1, g0 + DT - 1) / per_img) / imgs_per_group;
  const bool lds_stats = a.stats && (one_group || gfirst == glast);
  float s[8], ss[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = ss[k] = 0.f;
  for (int gi = gt; gi < total && gt < lim; gi = LOOP ? gi + stride : total) {
    const int c8 = gi % C8;
    int r = gi / C8;
    const int qs = r % QS;
    r /= QS;
    const int p = (r % PR) * DH, n = r / PR;      // first output row of this thread
    float wr[9][8];
    load_w72(a.w, c8, wr);
    constexpr int NCOL = (DWL - 1) * S + 3;
    const int q0 = qs * DWL, w0 = q0 * S - a.pad;
    // input prologue: this thread's 8 channels of its image's statistics group (same arithmetic
    // as bn.hip); NaN clamp bounds for act none keep NaN (conv_epi.h act_clamp_bounds)
    float psc[8], psh[8], plo = 0.f, phi = 0.f;
    if constexpr (PRO) {
      const int ch = c8 * 8;
      const float* m0p = a.pro_stats ? a.pro_stats + (size_t)(n / a.pro_group_imgs) * 2 * a.C + ch
                                     : a.pro_rmean + ch;
      const float* v0p = a.pro_stats ? m0p + a.C : a.pro_rvar + ch;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float mean = m0p[k], var = v0p[k];
        if (a.pro_stats) {
          mean *= a.pro_inv_count;
          var = fmaxf(var * a.pro_inv_count - mean * mean, 0.f);
        }
        psc[k] = a.pro_gamma[ch + k] * rsqrtf(var + a.pro_eps);
        psh[k] = a.pro_beta[ch + k] - mean * psc[k];
      }
      plo = a.pro_act == 0 ? __builtin_nanf("") : 0.f;
      phi = a.pro_act == 2 ? 6.f : (a.pro_act == 0 ? __builtin_nanf("") : __builtin_huge_valf());
    }
    float acc[DH][DWL][8];
#pragma unroll
    for (int d = 0; d < DH; ++d)
#pragma unroll
      for (int o = 0; o < DWL; ++o)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[d][o][k] = 0.f;
#pragma unroll
    for (int rr = 0; rr < (DH - 1) * S + 3; ++rr) {
      const int h = p * S - a.pad + rr;
      if (h >= 0 && h < a.H) {
        const bf16* row = a.x + (size_t)(n * a.H + h) * a.W * a.C + c8 * 8;
        bf16x8 col[NCOL];
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          const int ww = w0 + j;
          const bool in = ww >= 0 && ww < a.W;
          col[j] = ld8(row + (size_t)ww * a.C, in);
          if constexpr (PRO) {
            if (in) {
#pragma unroll
              for (int k = 0; k < 8; ++k)
                col[j][k] = f2bf(fminf(fmaxf(bf2f(col[j][k]) * psc[k] + psh[k], plo), phi));
              // the strip owning input (h, ww) writes the activation once: rows p*S ..
              // p*S+DH*S-1 (rr >= pad), columns of its own output strip
              if (a.keep && rr >= a.pad && rr < a.pad + DH * S && j >= a.pad && j < a.pad + DWL * S)
                *(bf16x8*)(a.keep + (size_t)(n * a.H + h) * a.W * a.C + (size_t)ww * a.C + c8 * 8) = col[j];
            }
          }
        }
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          const int kr = rr - d * S;                   // this input row's kernel row for output row d
          if (kr < 0 || kr > 2) continue;              // (compile-time after unrolling)
#pragma unroll
          for (int o = 0; o < DWL; ++o)
#pragma unroll
            for (int t = 0; t < 3; ++t)
#pragma unroll
              for (int k = 0; k < 8; ++k)
                acc[d][o][k] += bf2f(col[o * S + t][k]) * wr[kr * 3 + t][k];
        }
      }
    }
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      if (p + d >= a.P) break;
      bf16* yrow = a.y + (size_t)(n * a.P + p + d) * a.Q * a.C + c8 * 8;
#pragma unroll
      for (int o = 0; o < DWL; ++o) {
        if (q0 + o < a.Q) {
          bf16x8 v;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            v[k] = f2bf(acc[d][o][k]);
            const float f = bf2f(v[k]);
            s[k] += f;
            ss[k] += f * f;
          }
          *(bf16x8*)(yrow + (size_t)(q0 + o) * a.C) = v;
        }
      }
    }
    if (a.stats && !lds_stats) {  // block straddles two BN groups (tiny images): global atomics
      float* dst = MA_SPREAD(a.stats + (size_t)(n / imgs_per_group) * 2 * a.C);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        atomicAdd(dst + c8 * 8 + k, s[k]);
        atomicAdd(dst + a.C + c8 * 8 + k, ss[k]);
      }
    }
  }
  if (lds_stats) {
    // block reduction without LDS atomics: each thread's sums in its own padded LDS row, then
    // per channel over the threads of that channel's chunk (j0, j0 + C8, ...; gt = g0 + j)
    float* mine = part + threadIdx.x * ST_LD;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mine[k] = s[k];
      mine[8 + k] = ss[k];
    }
    __syncthreads();
    const int nthr = min(DT, lim - g0), off = g0 % C8;
    float* dst = MA_SPREAD(a.stats + (size_t)gfirst * 2 * a.C);
    for (int c = threadIdx.x; c < a.C; c += DT) {
      const int j0 = ((c >> 3) - off + C8) % C8;
      float v0 = 0.f, v1 = 0.f;
      for (int j = j0; j < nthr; j += C8) {
        v0 += part[j * ST_LD + (c & 7)];
        v1 += part[j * ST_LD + 8 + (c & 7)];
      }
      if (v1 != 0.f) {  // sumsq == 0 <=> no (non-zero) output of this channel in the block
        atomicAdd(dst + c, v0);
        atomicAdd(dst + a.C + c, v1);
      }
    }
  }
}

MA_DEV float dw_mask(float out, int act) {       // (bn.hip act_mask)
  if (act == 1) return out > 0.f ? 1.f : 0.f;
  if (act == 2) return (out > 0.f && out < 6.f) ? 1.f : 0.f;
  return 1.f;
}

// BW: the dgrad also reduces the BN-backward sums of the BN feeding this conv (what
// bn_bwd_reduce would do in a separate pass over dx, out and y): dz = dx * act'(out),
// sums += (dz, dz * xhat), block-reduced through padded LDS rows, one atomic pair per channel.
// (body shared by the standalone launch and the dgrad + wgrad pair: block ``bid`` of ``nblk``)
template <int S, bool BW>
MA_DEV void dw_dgrad_body(const bf16* dy, const float* w, bf16* dx, int N, int H, int W, int C,
                          int P, int Q, int pad, const DwBw& bw, float* part, int bid, int nblk) {
  // part (BW): [DT][ST_LD] per-thread (sum dz, sum dz * xhat)
  const int C8 = C >> 3, WS = (W + DWL - 1) / DWL;
  const int total = N * H * WS * C8;
  const int gt = bid * DT + threadIdx.x;
  // BW: a capped grid walks the strips (stride a multiple of C8: a thread keeps its channels),
  // so fewer blocks add their sums -- the per-channel atomics are what contends
  const int T = nblk * DT, stride = BW ? T - T % C8 : T;
  const int lim = min(total, stride);
  float sdz[8], sx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sdz[k] = sx[k] = 0.f;
  float wr[9][8];
  float mean[8], rstd[8];
  const int c8 = gt % C8;
  if (gt < lim) {
    load_w72(w, c8, wr);
    if constexpr (BW) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mean[k] = bw.stats[c8 * 8 + k] * bw.inv_count;
        rstd[k] = rsqrtf(fmaxf(bw.stats[C + c8 * 8 + k] * bw.inv_count - mean[k] * mean[k], 0.f) +
                         bw.eps);
      }
    }
  }
  for (int gi = gt; gi < total && gt < lim; gi += stride) {
    int r = gi / C8;
    const int ws = r % WS;
    r /= WS;
    const int h = r % H, n = r / H;
    const int x0 = ws * DWL;
    const size_t rowoff = (size_t)(n * H + h) * W * C + c8 * 8;
    // BW: the mask / BN-input chunks of the strip are requested with the dy loads
    bf16x8 ov[DWL], yv[DWL];
    if constexpr (BW) {
#pragma unroll
      for (int o = 0; o < DWL; ++o) {
        const bool in = x0 + o < W;
        ov[o] = ld8(bw.out + rowoff + (size_t)(x0 + o) * C, in);
        yv[o] = ld8(bw.y + rowoff + (size_t)(x0 + o) * C, in);
      }
    }
    float acc[DWL][8];
#pragma unroll
    for (int o = 0; o < DWL; ++o)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[o][k] = 0.f;
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      const int hp = h + pad - rr;
      if (S == 1) {
        if (hp >= 0 && hp < P) {
          const size_t roff = (size_t)(n * P + hp) * Q * C + c8 * 8;
          const bf16* row = dy + roff;
          bf16x8 col[DWL + 2];  // dy columns x0+pad-2 .. x0+DWL-1+pad
#pragma unroll
          for (int j = 0; j < DWL + 2; ++j) {
            const int q = x0 + pad - 2 + j;
            col[j] = ld8(row + (size_t)q * C, q >= 0 && q < Q);
          }
#pragma unroll
          for (int o = 0; o < DWL; ++o)
#pragma unroll
            for (int t = 0; t < 3; ++t)
#pragma unroll
              for (int k = 0; k < 8; ++k) acc[o][k] += bf2f(col[o + 2 - t][k]) * wr[rr * 3 + t][k];
        }
      } else {
        if (hp >= 0 && (hp % S) == 0 && hp / S < P) {
          const size_t roff = (size_t)(n * P + hp / S) * Q * C + c8 * 8;
          const bf16* row = dy + roff;
#pragma unroll
          for (int o = 0; o < DWL; ++o)
#pragma unroll
            for (int t = 0; t < 3; ++t) {
              const int wp = x0 + o + pad - t;
              if (wp >= 0 && (wp % S) == 0 && wp / S < Q) {
                const bf16x8 v = *(const bf16x8*)(row + (size_t)(wp / S) * C);
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[o][k] += bf2f(v[k]) * wr[rr * 3 + t][k];
              }
            }
        }
      }
    }
#pragma unroll
    for (int o = 0; o < DWL; ++o) {
      if (x0 + o < W) {
        bf16x8 v;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = f2bf(acc[o][k]);
        *(bf16x8*)(dx + rowoff + (size_t)(x0 + o) * C) = v;
        if constexpr (BW) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float dz = bf2f(v[k]) * dw_mask(bf2f(ov[o][k]), bw.act);
            sdz[k] += dz;
            sx[k] += dz * (bf2f(yv[o][k]) - mean[k]) * rstd[k];
          }
        }
      }
    }
  }
  if constexpr (BW) {
    float* mine = part + threadIdx.x * ST_LD;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mine[k] = sdz[k];
      mine[8 + k] = sx[k];
    }
    __syncthreads();
    const int g0 = bid * DT;
    const int nthr = min(DT, lim - g0), off = g0 % C8;
    for (int c = threadIdx.x; c < C; c += DT) {
      const int j0 = ((c >> 3) - off + C8) % C8;
      float v0 = 0.f, v1 = 0.f;
      for (int j = j0; j < nthr; j += C8) {
        v0 += part[j * ST_LD + (c & 7)];
        v1 += part[j * ST_LD + 8 + (c & 7)];
      }
      if (v0 != 0.f || v1 != 0.f) {     // replica blockIdx % SUMS_R of [SUMS_R][3][C]
        float* sums = bw.sums + (size_t)(bid % SUMS_R) * 3 * C;
        atomicAdd(sums + c, v0);
        atomicAdd(sums + C + c, v1);
      }
    }
  }
}

template <int S, bool BW>
__global__ __launch_bounds__(DT) void dw_dgrad_kernel(const bf16* dy, const float* w, bf16* dx, int N,
                                                      int H, int W, int C, int P, int Q, int pad,
                                                      DwBw bw) {
  extern __shared__ float part[];
  dw_dgrad_body<S, BW>(dy, w, dx, N, H, W, C, P, Q, pad, bw, part, blockIdx.x, gridDim.x);
}

// One thread per (image, output row, 8 channels) walks the row's columns with the 3x3 input
// window in registers, the next column's loads issued before the current column's FMAs.  The
// block then reduces its threads' 9x8 partial sums through LDS -- each thread's partials in
// its own padded LDS row, summed per (tap, channel) over the threads of that channel chunk --
// and adds 9C values into dw: no LDS atomics (the per-thread LDS atomic adds serialised on
// the ~256/C8 threads sharing a channel).
constexpr int WG_LD = 73;   // floats per thread row (odd: conflict-free row writes)
// A row is split into QS column segments of QL columns (one thread each): the serial walk --
// one memory round trip per column -- is QS x shorter and the grid QS x larger (the train-batch
// layers otherwise launch 48-100 blocks whose threads each walk 32 dependent columns).
template <int S>
MA_DEV void dw_wgrad_body(const bf16* dy, const bf16* x, float* dw, int N, int H, int W, int C,
                          int P, int Q, int pad, int QS, float* slab, float* part, int bid) {
  // part: [DT][WG_LD]
  const int C8 = C >> 3;
  const int total = N * P * QS * C8;
  const int QL = (Q + QS - 1) / QS;
  const int gt = bid * DT + threadIdx.x;
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[t][k] = 0.f;
  if (gt < total) {
    const int c8 = gt % C8;
    int r = gt / C8;
    const int seg = r % QS;
    r /= QS;
    const int p = r % P, n = r / P;
    const int q0 = seg * QL, q1 = min(q0 + QL, Q);
    const bf16* rows[3];
    bool rok[3];
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      const int h = p * S - pad + rr;
      rok[rr] = h >= 0 && h < H;
      rows[rr] = x + (size_t)(n * H + (rok[rr] ? h : 0)) * W * C + c8 * 8;
    }
    // sliding window win[rr][t] = x[h_rr][q*S - pad + t]
    bf16x8 win[3][3];
#pragma unroll
    for (int rr = 0; rr < 3; ++rr)
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int ww = q0 * S - pad + t;
        win[rr][t] = ld8(rows[rr] + (size_t)ww * C, q0 < q1 && rok[rr] && ww >= 0 && ww < W);
      }
    const size_t goff = (size_t)(n * P + p) * Q * C + c8 * 8;
    const bf16* grow = dy + goff;
    bf16x8 g = ld8(grow + (size_t)q0 * C, q0 < q1);
    for (int q = q0; q < q1; ++q) {
      // column q+1's loads first
      bf16x8 n1[3], n2[3], ng = g;
      const int base = (q + 1) * S - pad;
      const bool more = q + 1 < q1;
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        if (S == 2) n1[rr] = ld8(rows[rr] + (size_t)(base + 1) * C, more && rok[rr] && base + 1 >= 0 && base + 1 < W);
        n2[rr] = ld8(rows[rr] + (size_t)(base + 2) * C, more && rok[rr] && base + 2 >= 0 && base + 2 < W);
      }
      if (more) ng = *(const bf16x8*)(grow + (size_t)(q + 1) * C);
#pragma unroll
      for (int rr = 0; rr < 3; ++rr)
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[rr * 3 + t][k] += bf2f(g[k]) * bf2f(win[rr][t][k]);
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        if (S == 1) {
          win[rr][0] = win[rr][1];
          win[rr][1] = win[rr][2];
        } else {
          win[rr][0] = win[rr][2];
          win[rr][1] = n1[rr];
        }
        win[rr][2] = n2[rr];
      }
      g = ng;
    }
  }
  float* mine = part + threadIdx.x * WG_LD;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int k = 0; k < 8; ++k) mine[t * 8 + k] = acc[t][k];
  __syncthreads();
  // output (tap t, channel c): the threads of chunk c/8 are j0, j0 + C8, ... (gt = base + j)
  const int nthr = min(DT, total - bid * DT);   // (c8 stays the fastest index)
  const int off = (int)(((long long)bid * DT) % C8);
  for (int i = threadIdx.x; i < 9 * C; i += DT) {
    const int c = i % C, t = i / C;
    const int j0 = ((c >> 3) - off + C8) % C8;
    float v = 0.f;
    for (int j = j0; j < nthr; j += C8) v += part[j * WG_LD + t * 8 + (c & 7)];
    // slab: this block's partials, summed by dw_wgrad_reduce_kernel (no contended atomics)
    if (slab) slab[(size_t)bid * 9 * C + i] = v;
    else if (v != 0.f) atomicAdd(&dw[c * 9 + t], v);
  }
}

template <int S>
__global__ __launch_bounds__(DT) void dw_wgrad_kernel(const bf16* dy, const bf16* x, float* dw, int N,
                                                      int H, int W, int C, int P, int Q, int pad,
                                                      int QS, float* slab) {
  extern __shared__ float part[];
  dw_wgrad_body<S>(dy, x, dw, N, H, W, C, P, Q, pad, QS, slab, part, blockIdx.x);
}

// dgrad + wgrad of one depthwise conv in ONE launch (they read the same dy and are
// independent): blocks [0, nwg) are wgrad column segments, the rest dgrad strips
template <int S, bool BW>
__global__ __launch_bounds__(DT) void dw_bwd_kernel(const bf16* dy, const bf16* x, const float* w,
                                                    bf16* dx, float* dw, int N, int H, int W,
                                                    int C, int P, int Q, int pad, int QS,
                                                    float* slab, int nwg, DwBw bw) {
  extern __shared__ float part[];
  if ((int)blockIdx.x < nwg)
    dw_wgrad_body<S>(dy, x, dw, N, H, W, C, P, Q, pad, QS, slab, part, blockIdx.x);
  else
    dw_dgrad_body<S, BW>(dy, w, dx, N, H, W, C, P, Q, pad, bw, part, blockIdx.x - nwg,
                         gridDim.x - nwg);
}

// the partials reduce of several depthwise wgrads in one launch (blockIdx.z = layer): the
// train step defers every layer's reduce to the end of the backward
struct DwRedBatch {
  const float* slab[DW_RED_MAX];
  float* dw[DW_RED_MAX];
  int C[DW_RED_MAX], nblk[DW_RED_MAX];
};
__global__ __launch_bounds__(DT) void dw_wgrad_reduce_batch_kernel(DwRedBatch b) {
  const int l = blockIdx.z;
  const int C = b.C[l], nblk = b.nblk[l];
  if ((int)blockIdx.x * 64 >= 9 * C) return;          // whole block: this layer is narrower
  __shared__ float red[4][64];
  const int n9 = 9 * C;
  const int i = blockIdx.x * 64 + (threadIdx.x & 63), sub = threadIdx.x >> 6;
  const int share = (nblk + gridDim.y - 1) / gridDim.y;
  const int b0 = blockIdx.y * share, b1 = min(nblk, b0 + share);
  float v = 0.f;
  if (i < n9)
    for (int k = b0 + sub; k < b1; k += 4) v += b.slab[l][(size_t)k * n9 + i];
  red[sub][threadIdx.x & 63] = v;
  __syncthreads();
  if (sub == 0 && i < n9) {
    const float t = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    if (t != 0.f) atomicAdd(&b.dw[l][(i % C) * 9 + i / C], t);
  }
}

// dw[c][t] += sum over the wgrad blocks of their partials (slab [blocks][9][C], i = t*C + c).
// A block sums 64 outputs over a 1/gridDim.y share of the partials (4 sub-shares per output,
// reduced in LDS), then one atomic per output: gridDim.y-way instead of blocks-way contention,
// and a short (blocks / (4 gridDim.y)) load chain per thread.
__global__ __launch_bounds__(DT) void dw_wgrad_reduce_kernel(const float* slab, float* dw, int C,
                                                             int nblk) {
  __shared__ float red[4][64];
  const int n9 = 9 * C;
  const int i = blockIdx.x * 64 + (threadIdx.x & 63), sub = threadIdx.x >> 6;
  const int share = (nblk + gridDim.y - 1) / gridDim.y;
  const int b0 = blockIdx.y * share, b1 = min(nblk, b0 + share);
  float v = 0.f;
  if (i < n9)
    for (int b = b0 + sub; b < b1; b += 4) v += slab[(size_t)b * n9 + i];
  red[sub][threadIdx.x & 63] = v;
  __syncthreads();
  if (sub == 0 && i < n9) {
    const float t = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    if (t != 0.f) atomicAdd(&dw[(i % C) * 9 + i / C], t);
  }
}
}  // namespace

// blocks of the statistics-adding depthwise launches (every block's per-channel atomics land on
// the same few cache lines: fewer adders, less same-address serialisation at the memory side);
// MERCURY_DW_STAT_BLOCKS overrides for A/B runs
int dw_stat_blocks() {
  static const int v = [] {
    const char* e = getenv("MERCURY_DW_STAT_BLOCKS");
    const int x = e ? atoi(e) : 0;
    return x > 0 ? x : 256;
  }();
  return v;
}

// output rows per thread of the forward: 2 for the stride-1 convs of a large batch (the scoring
// pass, B = 320: 96 @32 96 -> 82 us, 144 @32 146 -> 119, 384 @8 31 -> 23), 1 elsewhere (at the
// B = 32 train batch the halved thread count cost 47 us over the chain, and the stride-2 convs
// at 16 / 8 wide lost 6 us each; bench/dw_stats_bench.py, profiles/r6/dw_dh/).  MERCURY_DW_DH=1/2
// forces one (A/B runs)
static int dw_dh(const DwArgs& a) {
  static const int force = [] {
    const char* e = getenv("MERCURY_DW_DH");
    return e ? atoi(e) : 0;
  }();
  if (force == 1 || force == 2) return force;
  return a.stride == 1 && a.N >= 128 ? 2 : 1;
}

void dwconv_fwd_launch(const DwArgs& a, hipStream_t st) {
  const int QS = (a.Q + DWL - 1) / DWL;
  const int DHr = dw_dh(a);
  const long long total = (long long)a.N * ((a.P + DHr - 1) / DHr) * QS * (a.C / 8);
  long long blocks = (total + DT - 1) / DT;
  // one statistics group: at most ~one block per CU adds the BN sums (grid-stride kernel)
  const int cap = dw_stat_blocks();
  const bool loop = a.stats && a.group_rows / (a.P * a.Q) >= a.N && blocks > cap;
  if (loop) blocks = cap;
  const dim3 grid((unsigned)blocks);
  const size_t shm = a.stats ? (size_t)DT * ST_LD * sizeof(float) : 0;
  const bool pro = a.pro_gamma != nullptr;
#define DW_FWD(S_, P_, L_)                                                                       \
  do {                                                                                           \
    if (DHr == 2) hipLaunchKernelGGL((dw_fwd_kernel<S_, P_, L_, 2>), grid, dim3(DT), shm, st, a); \
    else hipLaunchKernelGGL((dw_fwd_kernel<S_, P_, L_, 1>), grid, dim3(DT), shm, st, a);          \
  } while (0)
#define DW_FWD_L(S_, P_) \
  if (loop) DW_FWD(S_, P_, true); \
  else DW_FWD(S_, P_, false)
  if (a.stride == 1) {
    if (pro) DW_FWD_L(1, true);
    else DW_FWD_L(1, false);
  } else {
    if (pro) DW_FWD_L(2, true);
    else DW_FWD_L(2, false);
  }
#undef DW_FWD_L
#undef DW_FWD
}
void dwconv_dgrad_launch(const bf16* dy, const float* w, bf16* dx, int N, int H, int W, int C, int P,
                         int Q, int stride, int pad, hipStream_t st, const DwBw* bw) {
  const long long total = (long long)N * H * ((W + DWL - 1) / DWL) * (C / 8);
  // BW: at most ~one block per CU (each adds 2C atomics; C8 <= DT keeps a block's chunks whole)
  long long blocks = (total + DT - 1) / DT;
  if (bw && blocks > dw_stat_blocks()) blocks = dw_stat_blocks();
  const dim3 grid((unsigned)blocks);
  const DwBw none{};
  const size_t shm = bw ? (size_t)DT * ST_LD * sizeof(float) : 0;
#define DW_DG(S_, BW_) hipLaunchKernelGGL((dw_dgrad_kernel<S_, BW_>), grid, dim3(DT), shm, st, dy, w, \
                                          dx, N, H, W, C, P, Q, pad, bw ? *bw : none)
  if (stride == 1) {
    if (bw) DW_DG(1, true);
    else DW_DG(1, false);
  } else {
    if (bw) DW_DG(2, true);
    else DW_DG(2, false);
  }
#undef DW_DG
}
// wgrad column segments per row (QS) for the train-batch slab path
static int dw_qs(int N, int P, int Q, int C) {
  const long long rows = (long long)N * P * (C / 8);
  int QS = 1;
  while (rows * QS < 256LL * 4 * 64 && (Q + 2 * QS - 1) / (2 * QS) >= 4) QS *= 2;
  return QS;
}

int dwconv_wgrad_blocks(int N, int P, int Q, int C) {
  const long long total = (long long)N * P * (C / 8) * dw_qs(N, P, Q, C);
  return (int)((total + DT - 1) / DT);
}

void dwconv_bwd_launch(const bf16* dy, const bf16* x, const float* w, bf16* dx, float* dw, int N,
                       int H, int W, int C, int P, int Q, int stride, int pad, float* slab,
                       const DwBw* bw, bool reduce, hipStream_t st) {
  const int QS = dw_qs(N, P, Q, C);
  const int nwg = dwconv_wgrad_blocks(N, P, Q, C);
  const long long dtotal = (long long)N * H * ((W + DWL - 1) / DWL) * (C / 8);
  long long ndg = (dtotal + DT - 1) / DT;
  if (bw && ndg > dw_stat_blocks()) ndg = dw_stat_blocks();
  const size_t shm = (size_t)DT * WG_LD * sizeof(float);   // >= the dgrad's [DT][ST_LD]
  static const bool attr = [] {
    const void* ks[] = {(const void*)dw_bwd_kernel<1, false>, (const void*)dw_bwd_kernel<1, true>,
                        (const void*)dw_bwd_kernel<2, false>, (const void*)dw_bwd_kernel<2, true>};
    for (const void* k : ks)
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  const DwBw none{};
  const dim3 grid((unsigned)(nwg + ndg));
#define DW_B(S_, BW_) hipLaunchKernelGGL((dw_bwd_kernel<S_, BW_>), grid, dim3(DT), shm, st, dy, x, \
                                         w, dx, dw, N, H, W, C, P, Q, pad, QS, slab, nwg,          \
                                         bw ? *bw : none)
  if (stride == 1) {
    if (bw) DW_B(1, true);
    else DW_B(1, false);
  } else {
    if (bw) DW_B(2, true);
    else DW_B(2, false);
  }
#undef DW_B
  if (reduce) {
    const int shares = nwg >= 128 ? 8 : (nwg >= 32 ? 4 : 1);
    hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((9 * C + 63) / 64, shares), dim3(DT), 0, st, slab,
                       dw, C, nwg);
  }
}

void dwconv_wgrad_reduce_batch_launch(const float* const* slabs, float* const* dws, const int* Cs,
                                      const int* nblks, int n, hipStream_t st) {
  for (int l0 = 0; l0 < n; l0 += DW_RED_MAX) {
    DwRedBatch b{};
    int cmax = 0, bmax = 0;
    const int m = n - l0 < DW_RED_MAX ? n - l0 : DW_RED_MAX;
    for (int j = 0; j < m; ++j) {
      b.slab[j] = slabs[l0 + j];
      b.dw[j] = dws[l0 + j];
      b.C[j] = Cs[l0 + j];
      b.nblk[j] = nblks[l0 + j];
      cmax = b.C[j] > cmax ? b.C[j] : cmax;
      bmax = b.nblk[j] > bmax ? b.nblk[j] : bmax;
    }
    const int shares = bmax >= 128 ? 8 : (bmax >= 32 ? 4 : 1);
    hipLaunchKernelGGL(dw_wgrad_reduce_batch_kernel, dim3((9 * cmax + 63) / 64, shares, m),
                       dim3(DT), 0, st, b);
  }
}

size_t dwconv_wgrad_slab_floats(int N, int P, int Q, int C) {
  return (size_t)dwconv_wgrad_blocks(N, P, Q, C) * 9 * C;
}

void dwconv_wgrad_launch(const bf16* dy, const bf16* x, float* dw, int N, int H, int W, int C, int P,
                         int Q, int stride, int pad, hipStream_t st, float* slab,
                         size_t slab_floats) {
  // column segments: enough threads for ~4 waves per CU, segments of >= 4 columns; with a slab
  // (>= dwconv_wgrad_slab_floats) the blocks' partials are summed by a second small kernel
  // instead of contended atomics (each of the 100s of blocks adds every (channel, tap))
  const long long rows = (long long)N * P * (C / 8);
  int QS = 1;
  if (slab && slab_floats >= dwconv_wgrad_slab_floats(N, P, Q, C))
    while (rows * QS < 256LL * 4 * 64 && (Q + 2 * QS - 1) / (2 * QS) >= 4) QS *= 2;
  else
    slab = nullptr;
  const long long total = rows * QS;
  const dim3 grid((unsigned)((total + DT - 1) / DT));
  const size_t shm = (size_t)DT * WG_LD * sizeof(float);   // 73 KB: above the 64 KB default
  static const bool attr = [] {
    (void)hipFuncSetAttribute((const void*)dw_wgrad_kernel<1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)dw_wgrad_kernel<2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  if (stride == 1)
    hipLaunchKernelGGL(dw_wgrad_kernel<1>, grid, dim3(DT), shm, st, dy, x, dw, N, H, W, C, P, Q, pad,
                       QS, slab);
  else
    hipLaunchKernelGGL(dw_wgrad_kernel<2>, grid, dim3(DT), shm, st, dy, x, dw, N, H, W, C, P, Q, pad,
                       QS, slab);
  if (slab) {
    const int shares = grid.x >= 128 ? 8 : (grid.x >= 32 ? 4 : 1);
    hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((9 * C + 63) / 64, shares), dim3(DT), 0, st, slab,
                       dw, C, (int)grid.x);
  }
}
