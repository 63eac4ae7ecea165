// Classifier head: global average pool + linear + (importance-weighted) cross-entropy.
//
// Score mode is the reference's presample loss (`pytorch_collab.py:101-102`,
// `F.cross_entropy(reduction='none')`): per-sample
// l_i = logsumexp(z_i) - z_i[y_i].  Train mode is K4: the IS-weighted loss
// mean_i(l_i / w_i) (`:133-145`) and its gradient
// dz_i = (softmax(z_i) - onehot(y_i)) / (B * w_i), written in the same launch,
// plus device-side meters (loss sum, sample count, correct count) so the hot
// loop never syncs for `.item()` (`util.py:226-231`).
//
// One workgroup per sample: the pooled feature vector and the logits stay in
// LDS; dot products are wave64 reductions.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace {
constexpr int NT = 256;

// Wide heads (ImageNet: 2048 -> 1000 at B = 1280) first run the pool and the FC as their own
// launches -- the per-sample dot products above would stream the whole fp32 weight matrix
// once per sample (10 GB of L2 traffic, ~0.9 ms) -- and this kernel then only does the loss.

// pooled[b][c] = mean over HW of act[b][hw][c], one thread per (sample, 8 channels)
__global__ __launch_bounds__(NT) void head_pool_kernel(const bf16* act, float* pooled, int B, int HW,
                                                       int C) {
  const int C8 = C >> 3;
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= B * C8) return;
  const int b = i / C8, c = (i - b * C8) * 8;
  const bf16* x = act + (size_t)b * HW * C + c;
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
#pragma unroll 7
  for (int hw = 0; hw < HW; ++hw) {
    const bf16x8 v = *(const bf16x8*)(x + (size_t)hw * C);
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += bf2f(v[k]);
  }
  const float inv = 1.f / (float)HW;
  float* o = pooled + (size_t)b * C + c;
  *(float4*)o = make_float4(s[0] * inv, s[1] * inv, s[2] * inv, s[3] * inv);
  *(float4*)(o + 4) = make_float4(s[4] * inv, s[5] * inv, s[6] * inv, s[7] * inv);
}

// the pool with the final BN (+ identity residual) + activation applied on the fly (HeadArgs
// bn_*; reference: the block output `pytorch_model.py:34-36` then avg_pool2d + flatten `:94-95`):
// one thread per (sample, 8 channels), the raw conv output and the residual read once, each
// element normalised exactly as bn_apply_kernel would (scale / shift from the ghost-group sums or
// the running statistics) but kept in fp32 up to the mean
// (four consecutive lanes split one (sample, 8 channels)'s pixels and add up with two xor
// shuffles: 4x the threads of a one-lane pool, which left a 320-sample head latency-bound)
__global__ __launch_bounds__(NT) void head_pool_bn_kernel(HeadArgs a) {
  const int C8 = a.C >> 3;
  const int t = blockIdx.x * NT + threadIdx.x;
  const int i = t >> 2, sub = t & 3;
  const bool live = i < a.B * C8;
  const int b = live ? i / C8 : 0, c = live ? (i - b * C8) * 8 : 0;
  float sc[8], sh[8];
  {
    float m8[8], v8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (a.bn_stats) {
        const float* st = a.bn_stats + (size_t)(b / a.bn_group_imgs) * 2 * a.C + c + k;
        m8[k] = st[0] * a.bn_inv_count;
        v8[k] = fmaxf(st[a.C] * a.bn_inv_count - m8[k] * m8[k], 0.f);
      } else {
        m8[k] = a.bn_rmean[c + k];
        v8[k] = a.bn_rvar[c + k];
      }
      sc[k] = a.bn_gamma[c + k] * rsqrtf(v8[k] + a.bn_eps);
      sh[k] = a.bn_beta[c + k] - m8[k] * sc[k];
    }
  }
  const float lo = a.bn_act ? 0.f : -3.4e38f, hi = a.bn_act == 2 ? 6.f : 3.4e38f;
  const bf16* x = a.act + (size_t)b * a.HW * a.C + c;
  const bf16* r = a.bn_res ? a.bn_res + (size_t)b * a.HW * a.C + c : nullptr;
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (live) {
#pragma unroll 2
    for (int hw = sub; hw < a.HW; hw += 4) {
      const bf16x8 v = *(const bf16x8*)(x + (size_t)hw * a.C);
      bf16x8 rv;
      if (r) rv = *(const bf16x8*)(r + (size_t)hw * a.C);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float u = bf2f(v[k]) * sc[k] + sh[k];
        if (r) u += bf2f(rv[k]);
        s[k] += fminf(fmaxf(u, lo), hi);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s[k] += __shfl_xor(s[k], 1, 64);
    s[k] += __shfl_xor(s[k], 2, 64);
  }
  if (!live || sub) return;
  const float inv = 1.f / (float)a.HW;
  float* o = a.pooled + (size_t)b * a.C + c;
  *(float4*)o = make_float4(s[0] * inv, s[1] * inv, s[2] * inv, s[3] * inv);
  *(float4*)(o + 4) = make_float4(s[4] * inv, s[5] * inv, s[6] * inv, s[7] * inv);
}

// fp32 tiled GEMM for the wide head, C[m][n] = sum_r A(m, r) * B(n, r) (+ bias[n]), exact fp32
// like the per-sample path: 64x64 output tile per block, 4x4 per thread, 16-deep r slices
// through LDS with the next slice's global loads in flight during the current slice's FMAs.
// AR / BR: the operand is contiguous along r (row-major [m][r]) -- else along m / n
// ([r][m]).  Uses:  logits = pooled . W^T (AR, BR);  dpooled = dlogits . W (AR, !BR);
// dW = dlogits^T . pooled (!AR, !BR).  OUT 0: fp32 C; 1: bf16 C * scale broadcast over HW
// spatial rows (the activation gradient of the average pool).
constexpr int LT = 64, LK = 64;
// one 64 (rows) x 64 (r) operand slice per block, 16 floats per thread.  RC: thread -> row tid/4,
// r (tid%4)*16..+15;  else r tid/16 + 16j (j < 4), rows (tid%16)*4..+3.  A whole 64-deep slice
// per barrier pair: the loop is latency-bound (one block per CU), so fewer, larger slices.
// element type of a head operand: fp32, or bf16 (activations / packed weights, read 8 bytes at
// a time and widened)
MA_DEV float4 ld4x(const float* q) { return *(const float4*)q; }
MA_DEV float4 ld4x(const bf16* q) {
  const bf16x4 v = *(const bf16x4*)q;
  return make_float4(bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3]));
}
MA_DEV float ld1x(const float* q) { return *q; }
MA_DEV float ld1x(const bf16* q) { return bf2f(*q); }

template <bool RC, typename T>
MA_DEV void tile_load(const T* p, int ld, int i0, int ni, int r0, int nr, int tid,
                      float4 (&v)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = RC ? i0 + (tid >> 2) : i0 + (tid & 15) * 4;
    const int r = RC ? r0 + (tid & 3) * 16 + j * 4 : r0 + (tid >> 4) + 16 * j;
    float e[4];
    if (RC) {
      const T* q = p + (size_t)(i < ni ? i : 0) * ld + r;
      if (i < ni && r + 3 < nr) {
        v[j] = ld4x(q);
        continue;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) e[t] = (i < ni && r + t < nr) ? ld1x(q + t) : 0.f;
    } else {
      const T* q = p + (size_t)(r < nr ? r : 0) * ld + i;
      if (r < nr && i + 3 < ni) {
        v[j] = ld4x(q);
        continue;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) e[t] = (r < nr && i + t < ni) ? ld1x(q + t) : 0.f;
    }
    v[j] = make_float4(e[0], e[1], e[2], e[3]);
  }
}
template <bool RC>
MA_DEV void tile_store(float (*T)[LT + 4], const float4 (&v)[4], int tid) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (RC) {
      const int i = tid >> 2, r = (tid & 3) * 16 + j * 4;
      T[r + 0][i] = v[j].x; T[r + 1][i] = v[j].y; T[r + 2][i] = v[j].z; T[r + 3][i] = v[j].w;
    } else {
      *(float4*)&T[(tid >> 4) + 16 * j][(tid & 15) * 4] = v[j];
    }
  }
}

// OUT 2: bf16 C (plain row-major [M][N], * scale).  TA / TB: operand element types.  Split-R
// (gridDim.z > 1, OUT 0 only): each z-slice adds its partial product into C atomically (C must
// be zeroed; slice 0 adds the bias).
template <bool AR, bool BR, int OUT, typename TA = float, typename TB = float>
__global__ __launch_bounds__(NT) void head_gemm_kernel(const TA* A, int lda, const TB* Bm,
                                                       int ldb, const float* bias, void* out,
                                                       int M, int N, int R, int HW, float scale) {
  __shared__ float As[LK][LT + 4], Bs[LK][LT + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.x * LT, n0 = blockIdx.y * LT;
  // split-R: this block's slice [rb0, rb1) of the reduction (whole LK steps)
  const int nz = gridDim.z, per = ((R + LK - 1) / LK + nz - 1) / nz * LK;
  const int rb0 = blockIdx.z * per, rb1 = min(R, rb0 + per);
  float4 ra[4], rb[4];
  tile_load<AR>(A, lda, m0, M, rb0, rb1, tid, ra);
  tile_load<BR>(Bm, ldb, n0, N, rb0, rb1, tid, rb);
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int r0 = rb0; r0 < rb1; r0 += LK) {
    tile_store<AR>(As, ra, tid);
    tile_store<BR>(Bs, rb, tid);
    __syncthreads();
    if (r0 + LK < rb1) {
      tile_load<AR>(A, lda, m0, M, r0 + LK, rb1, tid, ra);
      tile_load<BR>(Bm, ldb, n0, N, r0 + LK, rb1, tid, rb);
    }
#pragma unroll
    for (int kk = 0; kk < LK; ++kk) {
      const float4 x = *(const float4*)&As[kk][ty * 4];
      const float4 y = *(const float4*)&Bs[kk][tx * 4];
      const float xa[4] = {x.x, x.y, x.z, x.w}, yb[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += xa[i] * yb[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
    if (OUT == 0) {
      float* o = (float*)out;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + tx * 4 + j;
        if (n >= N) continue;
        const float v = acc[i][j] + (bias && blockIdx.z == 0 ? bias[n] : 0.f);
        if (nz > 1) atomicAdd(o + (size_t)m * N + n, v);
        else o[(size_t)m * N + n] = v;
      }
    } else if (OUT == 2) {
      bf16* o = (bf16*)out + (size_t)m * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + tx * 4 + j;
        if (n < N) o[n] = f2bf(acc[i][j] * scale);
      }
    } else {
      bf16* o = (bf16*)out + (size_t)m * HW * N;
      const int n = n0 + tx * 4;
      if (n + 3 < N) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = f2bf(acc[i][j] * scale);
        for (int hw = 0; hw < HW; ++hw) *(bf16x4*)(o + (size_t)hw * N + n) = v;
      } else {
        for (int j = 0; j < 4; ++j)
          if (n + j < N)
            for (int hw = 0; hw < HW; ++hw) o[(size_t)hw * N + n + j] = f2bf(acc[i][j] * scale);
      }
    }
  }
}

// FC sizes from which the GEMM path wins (ImageNet 1000 x 2048 does; the CIFAR-100 MobileNetV2
// head, 100 x 1280, is faster on the per-sample path: too few 64x64 tiles to fill the GPU)
constexpr long long WIDE = 1ll << 20;

// db[k] = sum_b dlogits[b][k]
__global__ __launch_bounds__(NT) void head_db_kernel(const float* dlogits, float* db, int B, int K) {
  const int k = blockIdx.x * NT + threadIdx.x;
  if (k >= K) return;
  float s = 0.f;
#pragma unroll 16
  for (int b = 0; b < B; ++b) s += dlogits[(size_t)b * K + k];
  db[k] = s;
}

__global__ __launch_bounds__(NT) void head_fwd_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* pooled = sh;               // [C]
  float* logit = sh + a.C;          // [classes]
  float* red = logit + a.classes;   // [16]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (a.logits_ready) {
    if (a.score_kind == 1)
      for (int c = tid; c < a.C; c += NT) pooled[c] = a.pooled[(size_t)b * a.C + c];
    for (int k = tid; k < a.classes; k += NT) logit[k] = a.logits[(size_t)b * a.classes + k];
  } else {
    const bf16* x = a.act + (size_t)b * a.HW * a.C;
    const float invhw = 1.f / (float)a.HW;
    for (int c = tid; c < a.C; c += NT) {
      if (a.pooled_ready) {
        pooled[c] = a.pooled[(size_t)b * a.C + c];
        continue;
      }
      float s = 0.f;
#pragma unroll 8
      for (int hw = 0; hw < a.HW; ++hw) s += bf2f(x[(size_t)hw * a.C + c]);
      s *= invhw;
      pooled[c] = s;
      if (a.pooled) a.pooled[(size_t)b * a.C + c] = s;
    }
    __syncthreads();
    for (int k = wv; k < a.classes; k += NT / 64) {
      const float* wr = a.w + (size_t)k * a.C;
      float d = 0.f;
#pragma unroll 8
      for (int c = lane; c < a.C; c += 64) d += wr[c] * pooled[c];
      d = wave_sum(d);
      if (lane == 0) logit[k] = d + (a.b ? a.b[k] : 0.f);
    }
  }
  __syncthreads();
  // log-sum-exp and argmax, one wave
  if (wv == 0) {
    float mx = -3.4e38f;
    int am = 0;
    for (int k = lane; k < a.classes; k += 64) {
      if (logit[k] > mx) {
        mx = logit[k];
        am = k;
      }
    }
    // wave argmax (first max wins on ties, like torch.argmax)
    for (int o = 32; o >= 1; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oa < am)) {
        mx = om;
        am = oa;
      }
    }
    float se = 0.f;
    for (int k = lane; k < a.classes; k += 64) se += __expf(logit[k] - mx);
    se = wave_sum(se);
    const float lse = mx + __logf(se);
    const int y = a.label[b];
    const float loss = lse - logit[y];
    float score = loss;
    if (a.score_kind == 1) {
      // exact per-sample gradient norm of the classifier layer: d(loss)/d[W|b] is the outer
      // product of dz = softmax - onehot with [h, 1], so its Frobenius norm factorises
      float g2 = 0.f, h2 = 0.f;
      for (int k = lane; k < a.classes; k += 64) {
        const float d = __expf(logit[k] - lse) - (k == y ? 1.f : 0.f);
        g2 += d * d;
      }
      for (int c = lane; c < a.C; c += 64) h2 += pooled[c] * pooled[c];
      score = sqrtf(wave_sum(g2) * (wave_sum(h2) + 1.f));
    }
    if (lane == 0) {
      if (a.losses) a.losses[b] = score;
      red[0] = lse;
      const float wi = a.isw ? a.isw[b] : 1.f;
      if (a.mode == 1 || a.mode == 2) {
        if (a.meters) {
          atomicAdd(&a.meters[0], a.mode == 1 ? loss / wi : loss);
          atomicAdd(&a.meters[1], 1.f);
          atomicAdd(&a.meters[2], am == y ? 1.f : 0.f);
        }
      }
      red[1] = 1.f / ((float)a.B * wi);
    }
  }
  __syncthreads();
  if (a.mode == 1 && a.dlogits) {
    const float lse = red[0], scale = red[1];
    const int y = a.label[b];
    for (int k = tid; k < a.classes; k += NT) {
      const float p = __expf(logit[k] - lse);
      a.dlogits[(size_t)b * a.classes + k] = (p - (k == y ? 1.f : 0.f)) * scale;
    }
  }
}

// Narrow heads with many classes (MobileNetV2 CIFAR-100: 100 x 1280): the per-sample kernel's
// classes are a serial chain per wave (25 dot products of 1280 each); here block (b, j) pools
// sample b (redundantly per class chunk -- a few KB) and computes HC_CHUNK classes, so the
// chunks run as separate blocks; the loss / softmax kernel then runs on the ready logits.
constexpr int HC_CHUNK = 16;

MA_DEV void bn_act_bounds_h(int act, float& lo, float& hi) {   // (conv_epi.h bn_act_bounds)
  lo = act == 0 ? -__builtin_huge_valf() : 0.f;
  hi = act == 2 ? 6.f : __builtin_huge_valf();
}
__global__ __launch_bounds__(NT) void head_fc_chunk_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  float* pooled = sh;               // [C]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int k0 = blockIdx.y * HC_CHUNK;
  const bf16* x = a.act + (size_t)b * a.HW * a.C;
  const float invhw = 1.f / (float)a.HW;
  for (int c = tid; c < a.C; c += NT) {
    if (a.pooled_ready) {
      pooled[c] = a.pooled[(size_t)b * a.C + c];
      continue;
    }
    float s = 0.f;
#pragma unroll 8
    for (int hw = 0; hw < a.HW; ++hw) s += bf2f(x[(size_t)hw * a.C + c]);
    s *= invhw;
    pooled[c] = s;
    if (a.pooled && blockIdx.y == 0) a.pooled[(size_t)b * a.C + c] = s;
  }
  __syncthreads();
  const int k1 = min(a.classes, k0 + HC_CHUNK);
  for (int k = k0 + wv; k < k1; k += NT / 64) {
    const float* wr = a.w + (size_t)k * a.C;
    float d = 0.f;
#pragma unroll 8
    for (int c = lane; c < a.C; c += 64) d += wr[c] * pooled[c];
    d = wave_sum(d);
    if (lane == 0) a.logits[(size_t)b * a.classes + k] = d + (a.b ? a.b[k] : 0.f);
  }
}

// grid = (channel blocks, B + classes): block row y < B writes sample y's activation
// gradient (d pooled / HW broadcast over the spatial positions); row B + k reduces
// dW[k][:] (and db[k]) over the batch.  Every thread's loop is short and unrolled so
// its loads are in flight together.
__global__ __launch_bounds__(NT) void head_bwd_kernel(HeadBwdArgs a) {
  const int c = blockIdx.x * NT + threadIdx.x;
  const int b = blockIdx.y;
  if (b >= a.B) {
    const int k = b - a.B;
    if (blockIdx.x == 0 && threadIdx.x < 64) {
      float s = 0.f;
      for (int i = threadIdx.x; i < a.B; i += 64) s += a.dlogits[(size_t)i * a.classes + k];
      s = wave_sum(s);
      if (threadIdx.x == 0) a.db[k] = s;
    }
    if (c >= a.C) return;
    float s = 0.f;
#pragma unroll 8
    for (int i = 0; i < a.B; ++i)
      s += a.dlogits[(size_t)i * a.classes + k] * a.pooled[(size_t)i * a.C + c];
    a.dw[(size_t)k * a.C + c] = s;
    return;
  }
  if (c >= a.C) return;
  float s = 0.f;
#pragma unroll 8
  for (int k = 0; k < a.classes; ++k)
    s += a.dlogits[(size_t)b * a.classes + k] * a.w[(size_t)k * a.C + c];
  const bf16 v = f2bf(s / (float)a.HW);
  bf16* dst = a.dact + (size_t)b * a.HW * a.C + c;
#pragma unroll 8
  for (int hw = 0; hw < a.HW; ++hw) dst[(size_t)hw * a.C] = v;
  if (a.bw_sums != nullptr) {
    // the final BN's backward sums over this sample's HW positions of channel c (the reduce
    // pass bn_bwd would otherwise make): same arithmetic as the dgrad epilogue
    float lo, hi;
    bn_act_bounds_h(a.bw_act, lo, hi);
    const bool pass = a.bw_act == 0;
    const float m1 = a.bw_stats[c] * a.bw_inv_count;
    const float r1 = rsqrtf(fmaxf(a.bw_stats[a.C + c] * a.bw_inv_count - m1 * m1, 0.f) + a.bw_eps);
    float m2 = 0.f, r2 = 0.f;
    if (a.bw_y2) {
      m2 = a.bw_stats2[c] * a.bw_inv_count;
      r2 = rsqrtf(fmaxf(a.bw_stats2[a.C + c] * a.bw_inv_count - m2 * m2, 0.f) + a.bw_eps);
    }
    const float g = bf2f(v);
    const size_t base = (size_t)b * a.HW * a.C + c;
    float sdz = 0.f, sx = 0.f, sx2 = 0.f;
    // 8 positions' loads issued before their math: the rolled loop waited out one memory
    // latency per position (11.6 us for ResNet-18's 4x4 head, profiles/r4/seq/seq_train.txt)
    constexpr int U = 8;
    const bool two = a.bw_y2 != nullptr;
    for (int h0 = 0; h0 < a.HW; h0 += U) {
      float ov[U], yv[U], y2v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int hw = min(h0 + u, a.HW - 1);
        const size_t o = base + (size_t)hw * a.C;
        ov[u] = bf2f(a.bw_out[o]);
        yv[u] = bf2f(a.bw_y[o]);
        y2v[u] = two ? bf2f(a.bw_y2[o]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (h0 + u >= a.HW) break;             // uniform: HW is a kernel argument
        const float dz = (pass || (ov[u] > lo && ov[u] < hi)) ? g : 0.f;
        sdz += dz;
        sx += dz * (yv[u] - m1) * r1;
        if (two) sx2 += dz * (y2v[u] - m2) * r2;
      }
    }
    float* sums = a.bw_sums + (size_t)(b % SUMS_R) * 3 * a.C;
    atomicAdd(sums + c, sdz);
    atomicAdd(sums + a.C + c, sx);
    if (a.bw_y2) atomicAdd(sums + 2 * a.C + c, sx2);
  }
}
}  // namespace

void head_fwd_launch(const HeadArgs& a0, hipStream_t st) {
  HeadArgs a = a0;
  a.logits_ready = 0;
  static const int path = [] {
    const char* v = getenv("MERCURY_HEAD_PATH");   // (A/B: 0 auto, 1 per-sample, 2 pool + GEMM)
    return v ? atoi(v) : 0;
  }();
  const bool wide = path == 2 || (path == 0 && (long long)a.classes * a.C >= WIDE);
  // wide heads: pool + fp32 tiled FC as their own launches (needs the pooled/logits workspaces);
  // the FC reduction is split over the channels so the launch fills the GPU (slices add into
  // the zeroed logits)
  if (a.bn_gamma) {
    // the final BN (+ residual) + activation in the pool: pooled[] first, then the FC
    hipLaunchKernelGGL(head_pool_bn_kernel, dim3((4 * a.B * (a.C / 8) + NT - 1) / NT), dim3(NT),
                       0, st, a);
    a.pooled_ready = 1;
  }
  if (wide && a.pooled && a.logits && a.C % 16 == 0) {
    if (!a.pooled_ready)
      hipLaunchKernelGGL(head_pool_kernel, dim3((a.B * (a.C / 8) + NT - 1) / NT), dim3(NT), 0, st,
                         a.act, a.pooled, a.B, a.HW, a.C);
    const int tiles = ((a.B + LT - 1) / LT) * ((a.classes + LT - 1) / LT);
    int z = 1;
    while (tiles * z * 2 <= 256 && a.C / (z * 2) >= 4 * LK) z *= 2;
    if (z > 1) (void)hipMemsetAsync(a.logits, 0, sizeof(float) * a.B * a.classes, st);
    hipLaunchKernelGGL((head_gemm_kernel<true, true, 0>),
                       dim3((a.B + LT - 1) / LT, (a.classes + LT - 1) / LT, z), dim3(NT), 0, st,
                       a.pooled, a.C, a.w, a.C, a.b, (void*)a.logits, a.B, a.classes, a.C, 1, 1.f);
    a.logits_ready = 1;
  } else if (path != 1 && a.logits && a.classes >= 4 * HC_CHUNK) {
    hipLaunchKernelGGL(head_fc_chunk_kernel, dim3(a.B, (a.classes + HC_CHUNK - 1) / HC_CHUNK),
                       dim3(NT), (size_t)a.C * sizeof(float), st, a);
    a.logits_ready = 1;
  }
  const size_t shm = (size_t)(a.C + a.classes + 16) * sizeof(float);
  hipLaunchKernelGGL(head_fwd_kernel, dim3(a.B), dim3(NT), shm, st, a);
}

// ---------------------------------------------------------------- speech-VGG head
// flatten -> fc1 -> fc2 -> log_softmax (`pytorch_model.py:145-153`).  fc1's weights are kept
// in the engine's [f1][H][W][C] layout (the flatten order of an NHWC activation; torch's
// [f1][C][H][W] at the state-dict boundary), so fc1 is a plain GEMM on the activation rows.
// Forward: h1 = x . W1^T + b1 (split-R, atomics into a zeroed h1), logits = h1 . W2^T + b2, then
// the loss / dlogits / meters kernel.  Backward: dW2, db2, dh1 = dlogits . W2, db1, dW1 =
// dh1^T . x (straight into the flat gradient, engine layout), dx = dh1 . W1 (bf16 NHWC).
void mlp_head_fwd_launch(const bf16* x, const bf16* w1, const float* b1, const float* w2,
                         const float* b2, float* h1, float* logits, int B, int F, int H1, int K,
                         int splits, hipStream_t st) {
  (void)hipMemsetAsync(h1, 0, sizeof(float) * B * H1, st);
  hipLaunchKernelGGL((head_gemm_kernel<true, true, 0, bf16, bf16>),
                     dim3((B + LT - 1) / LT, (H1 + LT - 1) / LT, splits), dim3(NT), 0, st, x, F,
                     w1, F, b1, (void*)h1, B, H1, F, 1, 1.f);
  hipLaunchKernelGGL((head_gemm_kernel<true, true, 0>), dim3((B + LT - 1) / LT, (K + LT - 1) / LT),
                     dim3(NT), 0, st, h1, H1, w2, H1, b2, (void*)logits, B, K, H1, 1, 1.f);
}

void mlp_head_bwd_launch(const float* dlogits, const float* h1, const bf16* x, const bf16* w1,
                         const float* w2, float* dh1, float* dw1, float* db1, float* dw2,
                         float* db2, bf16* dx, int B, int F, int H1, int K, hipStream_t st) {
  hipLaunchKernelGGL((head_gemm_kernel<false, false, 0>), dim3((K + LT - 1) / LT, (H1 + LT - 1) / LT),
                     dim3(NT), 0, st, dlogits, K, h1, H1, (const float*)nullptr, (void*)dw2, K,
                     H1, B, 1, 1.f);
  hipLaunchKernelGGL(head_db_kernel, dim3((K + NT - 1) / NT), dim3(NT), 0, st, dlogits, db2, B, K);
  hipLaunchKernelGGL((head_gemm_kernel<true, false, 0>), dim3((B + LT - 1) / LT, (H1 + LT - 1) / LT),
                     dim3(NT), 0, st, dlogits, K, w2, H1, (const float*)nullptr, (void*)dh1, B, H1,
                     K, 1, 1.f);
  hipLaunchKernelGGL(head_db_kernel, dim3((H1 + NT - 1) / NT), dim3(NT), 0, st, dh1, db1, B, H1);
  hipLaunchKernelGGL((head_gemm_kernel<false, false, 0, float, bf16>),
                     dim3((H1 + LT - 1) / LT, (F + LT - 1) / LT), dim3(NT), 0, st, dh1, H1, x, F,
                     (const float*)nullptr, (void*)dw1, H1, F, B, 1, 1.f);
  hipLaunchKernelGGL((head_gemm_kernel<true, false, 2, float, bf16>),
                     dim3((B + LT - 1) / LT, (F + LT - 1) / LT), dim3(NT), 0, st, dh1, H1, w1, F,
                     (const float*)nullptr, (void*)dx, B, F, H1, 1, 1.f);
}

// loss / dlogits / meters / score from precomputed logits (a.pooled: the classifier input, for
// the gradient-norm score)
void head_loss_launch(const HeadArgs& a0, hipStream_t st) {
  HeadArgs a = a0;
  a.logits_ready = 1;
  const size_t shm = (size_t)(a.C + a.classes + 16) * sizeof(float);
  hipLaunchKernelGGL(head_fwd_kernel, dim3(a.B), dim3(NT), shm, st, a);
}

int head_bwd_launch(const HeadBwdArgs& a, hipStream_t st) {
  if ((long long)a.classes * a.C >= WIDE && a.classes % 4 == 0 && a.C % 4 == 0) {
    // wide head: dact = (dlogits . W) / HW broadcast over HW, dW = dlogits^T . pooled, db
    hipLaunchKernelGGL((head_gemm_kernel<true, false, 1>),
                       dim3((a.B + LT - 1) / LT, (a.C + LT - 1) / LT), dim3(NT), 0, st,
                       a.dlogits, a.classes, a.w, a.C, (const float*)nullptr, (void*)a.dact, a.B,
                       a.C, a.classes, a.HW, 1.f / (float)a.HW);
    hipLaunchKernelGGL((head_gemm_kernel<false, false, 0>),
                       dim3((a.classes + LT - 1) / LT, (a.C + LT - 1) / LT), dim3(NT), 0, st,
                       a.dlogits, a.classes, a.pooled, a.C, (const float*)nullptr, (void*)a.dw,
                       a.classes, a.C, a.B, 1, 1.f);
    hipLaunchKernelGGL(head_db_kernel, dim3((a.classes + NT - 1) / NT), dim3(NT), 0, st,
                       a.dlogits, a.db, a.B, a.classes);
    return 0;
  }
  hipLaunchKernelGGL(head_bwd_kernel, dim3((a.C + NT - 1) / NT, a.B + a.classes), dim3(NT), 0, st,
                     a);
  return a.bw_sums != nullptr;
}
