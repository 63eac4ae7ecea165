// Direct-xGMI two-shot all-reduce: the GPU counterpart of the reference's
// hand-written CPU ring (`util.py:280-324`), designed for MI355X's fully connected xGMI
// (7 point-to-point links per GPU, ~153 GB/s each) instead of a ring.
//
// A ring all-reduce moves every byte over ONE link per step, so on an 8-GPU node it uses 2 of
// the 7 links of each GPU.  Here every rank has an exchange buffer that every peer maps with
// hipIpcOpenMemHandle, and the reduction is two direct passes:
//
//   reduce-scatter : rank r owns chunk r (n / W elements, 16-byte aligned); one kernel reads
//                    chunk r from ALL W exchange buffers at once (W-1 of them remote: all 7
//                    links busy in parallel), sums in fp32 and writes the result into chunk r
//                    of its own exchange buffer;
//   all-gather     : one kernel reads chunk p of peer p's exchange buffer for every p and
//                    writes the full reduced vector into the local destination.
//
// Each rank moves 2 (W-1)/W n elements over xGMI -- the same as a ring -- but spread over
// W-1 links instead of one.  The passes are separated by stream-ordered barriers (a one-
// element RCCL all-reduce on the same stream, or a host barrier in tests), so the kernels
// themselves need no cross-GPU flags.  ``wire_bf16``: the exchange buffers hold bf16 (half the
// bytes over the links); sums are accumulated in fp32 and rounded once per pass.
//
// For testing on one GPU the "peers" are simply W local buffers (emulated ranks).
#include <algorithm>
#include <string>

#include "common.h"

namespace {

constexpr int XMAX = 8;

struct Peers {
  const void* p[XMAX];
};

MA_DEV f32x4 ld4(const void* base, long long i, bool bf) {
  if (!bf) return ((const f32x4*)base)[i];
  const bf16* b = (const bf16*)base + i * 4;
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  const bf16x4_t v = *(const bf16x4_t*)b;
  return f32x4{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
}

MA_DEV void st4(void* base, long long i, f32x4 v, bool bf) {
  if (!bf) {
    ((f32x4*)base)[i] = v;
    return;
  }
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  bf16x4_t o;
  o[0] = f2bf(v[0]);
  o[1] = f2bf(v[1]);
  o[2] = f2bf(v[2]);
  o[3] = f2bf(v[3]);
  *(bf16x4_t*)((bf16*)base + i * 4) = o;
}

// chunk r = [off(r), off(r+1)) in float4 units
__host__ __device__ inline long long chunk_off(long long n4, int W, int r) { return r >= W ? n4 : n4 * r / W; }

template <bool BF>
__global__ __launch_bounds__(256) void xgmi_rs_kernel(Peers peers, int W, int rank, long long n4,
                                                      float scale) {
  const long long c0 = chunk_off(n4, W, rank), c1 = chunk_off(n4, W, rank + 1);
  for (long long i = c0 + (long long)blockIdx.x * 256 + threadIdx.x; i < c1;
       i += (long long)gridDim.x * 256) {
    f32x4 acc = ld4(peers.p[0], i, BF);
#pragma unroll
    for (int q = 1; q < XMAX; ++q)
      if (q < W) acc += ld4(peers.p[q], i, BF);
    st4((void*)peers.p[rank], i, acc * scale, BF);
  }
}

// dst (fp32, local) <- chunk p of peer p, for every p
template <bool BF>
__global__ __launch_bounds__(256) void xgmi_ag_kernel(Peers peers, int W, long long n4,
                                                      float* __restrict__ dst) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (long long)gridDim.x * 256) {
    // owner of element i: the p with off(p) <= i < off(p+1)
    int p = (int)((i * W) / n4);
    while (p > 0 && chunk_off(n4, W, p) > i) --p;
    while (p + 1 < W && chunk_off(n4, W, p + 1) <= i) ++p;
    ((f32x4*)dst)[i] = ld4(peers.p[p], i, BF);
  }
}

__global__ __launch_bounds__(256) void xgmi_pack_kernel(const float* __restrict__ src,
                                                        void* __restrict__ xbuf, long long n4,
                                                        int bf) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4;
       i += (long long)gridDim.x * 256)
    st4(xbuf, i, ((const f32x4*)src)[i], bf != 0);
}

unsigned grid_for(long long n4) {
  long long b = (n4 + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

}  // namespace

// n: element count (a multiple of 4; the engine's buckets are 4-aligned flat ranges)
void xgmi_pack(const float* src, void* xbuf, long long n, int bf, hipStream_t st) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(xgmi_pack_kernel, dim3(grid_for(n4)), dim3(256), 0, st, src, xbuf, n4, bf);
}

void xgmi_reduce_scatter(const void* const* peers, int W, int rank, long long n, int bf,
                         float scale, hipStream_t st) {
  Peers p{};
  for (int q = 0; q < W && q < XMAX; ++q) p.p[q] = peers[q];
  const long long n4 = n / 4;
  const long long mine = chunk_off(n4, W, rank + 1) - chunk_off(n4, W, rank);
  if (bf)
    hipLaunchKernelGGL(xgmi_rs_kernel<true>, dim3(grid_for(mine)), dim3(256), 0, st, p, W, rank,
                       n4, scale);
  else
    hipLaunchKernelGGL(xgmi_rs_kernel<false>, dim3(grid_for(mine)), dim3(256), 0, st, p, W, rank,
                       n4, scale);
}

void xgmi_all_gather(const void* const* peers, int W, long long n, int bf, float* dst,
                     hipStream_t st) {
  Peers p{};
  for (int q = 0; q < W && q < XMAX; ++q) p.p[q] = peers[q];
  const long long n4 = n / 4;
  if (bf)
    hipLaunchKernelGGL(xgmi_ag_kernel<true>, dim3(grid_for(n4)), dim3(256), 0, st, p, W, n4, dst);
  else
    hipLaunchKernelGGL(xgmi_ag_kernel<false>, dim3(grid_for(n4)), dim3(256), 0, st, p, W, n4, dst);
}

int xgmi_max_ranks() { return XMAX; }

// IPC: export a device allocation / map a peer's (one process per GPU; HSA_ENABLE_IPC_MODE_LEGACY=0)
std::string xgmi_ipc_handle(uintptr_t ptr) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, (void*)ptr) != hipSuccess) return std::string();
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

uintptr_t xgmi_ipc_open(const std::string& handle) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) return 0;
  hipIpcMemHandle_t h;
  std::copy(handle.begin(), handle.end(), reinterpret_cast<char*>(&h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return 0;
  return reinterpret_cast<uintptr_t>(p);
}

uintptr_t xgmi_malloc(long long bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, (size_t)bytes) != hipSuccess) return 0;
  (void)hipMemset(p, 0, (size_t)bytes);
  return reinterpret_cast<uintptr_t>(p);
}

void xgmi_free(uintptr_t p) {
  if (p) (void)hipFree(reinterpret_cast<void*>(p));
}

void xgmi_ipc_close(uintptr_t p) {
  if (p) (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(p));
}
