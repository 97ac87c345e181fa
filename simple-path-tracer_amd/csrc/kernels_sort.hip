// kernels_sort.hip — the LBVH build's device primitives, written for gfx950 (wave64): a stable LSD
// radix sort of 64-bit keys with 32-bit values (the Morton codes of the primitive references) and an
// exclusive prefix sum of 32-bit counts (slot assignment, split-reference offsets, wide-level offsets).
// They replace the rocPRIM calls of r01-r03 (north_star: "on-device LBVH (Morton + radix sort)").
//
// Radix sort: 8 passes of 8-bit digits, least significant first.  A pass over a tile of
// kSortTile = 4096 keys per workgroup (256 threads x 16):
//   k_rs_hist    : the tile's digit histogram in LDS -> hist[digit * tiles + tile] (digit-major)
//   exclusive scan of hist (scan_u32) -> the global start of each (digit, tile) run
//   k_rs_scatter : each key goes to start[digit][tile] + its stable rank among the tile's keys of that
//                  digit.  The tile is walked in its own order, 256 keys per round; a key's rank is the
//                  count of its digit in the earlier rounds (s_run), in the round's earlier waves
//                  (s_wave), and in its own wave's lower lanes (an 8-ballot digit match).
// Stability of every pass makes the whole sort stable: equal keys keep their input order, so the
// result equals rocprim::radix_sort_pairs' (and a stable CPU sort's) element for element.
//
// Scan: tiles of kScanTile = 4096 counts — per-tile sums, an exclusive scan of the sums in one
// workgroup (looping over them), then each tile's exclusive scan from its sum's offset.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sptr_internal.h"

namespace sptr {

namespace {

constexpr uint32_t kSortBlock = 256;
constexpr uint32_t kSortItems = 16;
constexpr uint32_t kSortTile = kSortBlock * kSortItems;
constexpr uint32_t kRadix = 256;
constexpr uint32_t kScanTile = 4096;

__device__ __forceinline__ uint32_t digit_of(uint64_t k, uint32_t shift) { return (uint32_t)(k >> shift) & 0xFFu; }

__global__ void __launch_bounds__(kSortBlock) k_rs_hist(const uint64_t* keys, uint32_t n, uint32_t shift, uint32_t tiles,
                                                         uint32_t* hist) {
  __shared__ uint32_t s_h[kRadix];
  s_h[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t base = blockIdx.x * kSortTile;
#pragma unroll
  for (uint32_t j = 0; j < kSortItems; ++j) {
    const uint32_t i = base + j * kSortBlock + threadIdx.x;
    if (i < n) atomicAdd(&s_h[digit_of(keys[i], shift)], 1u);
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * tiles + blockIdx.x] = s_h[threadIdx.x];
}

__global__ void __launch_bounds__(kSortBlock) k_rs_scatter(const uint64_t* keys, const uint32_t* vals, uint32_t n,
                                                            uint32_t shift, uint32_t tiles, const uint32_t* start,
                                                            uint64_t* keys_out, uint32_t* vals_out) {
  __shared__ uint32_t s_start[kRadix];                     // this tile's first output slot of each digit
  __shared__ uint32_t s_run[kRadix];                       // keys of each digit in the tile's earlier rounds
  __shared__ uint32_t s_wave[kSortBlock / 64][kRadix];     // keys of each digit per wave of this round
  const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  s_start[threadIdx.x] = start[(size_t)threadIdx.x * tiles + blockIdx.x];
  s_run[threadIdx.x] = 0u;
  const uint32_t base = blockIdx.x * kSortTile;
  for (uint32_t j = 0; j < kSortItems; ++j) {
    for (uint32_t w = 0; w < kSortBlock / 64; ++w) s_wave[w][threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t i = base + j * kSortBlock + threadIdx.x;
    const bool ok = i < n;
    const uint64_t k = ok ? keys[i] : 0ull;
    const uint32_t v = ok ? vals[i] : 0u;
    const uint32_t d = digit_of(k, shift);
    // lanes of this wave holding the same digit
    unsigned long long same = __ballot(ok);
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
      const unsigned long long set = __ballot(ok && ((d >> b) & 1u));
      same &= ((d >> b) & 1u) ? set : ~set;
    }
    const uint32_t in_wave = (uint32_t)__popcll(same & below);
    // the lowest lane of each digit group publishes the group's count
    if (ok && in_wave == 0u) s_wave[wave][d] = (uint32_t)__popcll(same);
    __syncthreads();
    if (ok) {
      uint32_t r = s_run[d] + in_wave;
      for (uint32_t w = 0; w < wave; ++w) r += s_wave[w][d];
      const uint32_t dst = s_start[d] + r;
      keys_out[dst] = k;
      vals_out[dst] = v;
    }
    __syncthreads();
    uint32_t add = 0u;
    for (uint32_t w = 0; w < kSortBlock / 64; ++w) add += s_wave[w][threadIdx.x];
    s_run[threadIdx.x] += add;
  }
}

// ---- exclusive scan of u32 counts
__device__ __forceinline__ uint32_t block_exclusive(uint32_t x, uint32_t* s_w, uint32_t& total) {
  const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
  uint32_t incl = x;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off);
    if (lane >= (uint32_t)off) incl += y;
  }
  if (lane == 63u) s_w[wave] = incl;
  __syncthreads();
  uint32_t before = 0u;
  total = 0u;
  for (uint32_t w = 0; w < blockDim.x / 64u; ++w) {
    if (w < wave) before += s_w[w];
    total += s_w[w];
  }
  __syncthreads();
  return before + incl - x;
}
// per tile of kScanTile counts: its sum (each thread sums 16 consecutive counts)
__global__ void __launch_bounds__(kSortBlock) k_scan_sums(const uint32_t* in, uint32_t n, uint32_t* sums) {
  __shared__ uint32_t s_w[kSortBlock / 64];
  const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * 16u;
  uint32_t x = 0u;
#pragma unroll
  for (uint32_t j = 0; j < 16u; ++j) x += (base + j < n) ? in[base + j] : 0u;
  uint32_t total;
  (void)block_exclusive(x, s_w, total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}
// one workgroup: exclusive scan of the m tile sums in place
__global__ void __launch_bounds__(kSortBlock) k_scan_top(uint32_t* sums, uint32_t m) {
  __shared__ uint32_t s_w[kSortBlock / 64];
  uint32_t carry = 0u;
  for (uint32_t b = 0; b < m; b += kSortBlock) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t x = i < m ? sums[i] : 0u;
    uint32_t total;
    const uint32_t ex = block_exclusive(x, s_w, total);
    if (i < m) sums[i] = carry + ex;
    carry += total;
  }
}
__global__ void __launch_bounds__(kSortBlock) k_scan_tiles(const uint32_t* in, uint32_t n, const uint32_t* sums, uint32_t* out) {
  __shared__ uint32_t s_w[kSortBlock / 64];
  const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * 16u;
  uint32_t v[16];
  uint32_t x = 0u;
#pragma unroll
  for (uint32_t j = 0; j < 16u; ++j) {
    v[j] = (base + j < n) ? in[base + j] : 0u;
    x += v[j];
  }
  uint32_t total;
  uint32_t run = sums[blockIdx.x] + block_exclusive(x, s_w, total);
#pragma unroll
  for (uint32_t j = 0; j < 16u; ++j) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
}

inline size_t align256(size_t b) { return (b + 255u) / 256u * 256u; }

}  // namespace

// temp == nullptr: only set temp_bytes.  out may alias in.
hipError_t scan_u32(void* temp, size_t& temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s) {
  const uint32_t m = (n + kScanTile - 1u) / kScanTile;
  const size_t need = align256((size_t)(m ? m : 1u) * 4u);
  if (!temp) {
    temp_bytes = need;
    return hipSuccess;
  }
  if (temp_bytes < need) return hipErrorInvalidValue;
  if (n == 0u) return hipSuccess;
  uint32_t* sums = static_cast<uint32_t*>(temp);
  hipLaunchKernelGGL(k_scan_sums, dim3(m), dim3(kSortBlock), 0, s, in, n, sums);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kSortBlock), 0, s, sums, m);
  hipLaunchKernelGGL(k_scan_tiles, dim3(m), dim3(kSortBlock), 0, s, in, n, sums, out);
  return hipGetLastError();
}

// Stable ascending sort of (keys_in, vals_in) into (keys_out, vals_out); the inputs are not modified.
hipError_t radix_sort_pairs_u64(void* temp, size_t& temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                                const uint32_t* vals_in, uint32_t* vals_out, uint32_t n, hipStream_t s) {
  const uint32_t tiles = (n + kSortTile - 1u) / kSortTile;
  const uint32_t hn = kRadix * (tiles ? tiles : 1u);
  size_t scan_bytes = 0;
  (void)scan_u32(nullptr, scan_bytes, nullptr, nullptr, hn, s);
  const size_t kb = align256((size_t)(n ? n : 1u) * 8u), vb = align256((size_t)(n ? n : 1u) * 4u),
               hb = align256((size_t)hn * 4u);
  const size_t need = kb + vb + 2u * hb + scan_bytes;
  if (!temp) {
    temp_bytes = need;
    return hipSuccess;
  }
  if (temp_bytes < need) return hipErrorInvalidValue;
  if (n == 0u) return hipSuccess;
  char* t = static_cast<char*>(temp);
  uint64_t* kt = reinterpret_cast<uint64_t*>(t);
  uint32_t* vt = reinterpret_cast<uint32_t*>(t + kb);
  uint32_t* hist = reinterpret_cast<uint32_t*>(t + kb + vb);
  uint32_t* start = reinterpret_cast<uint32_t*>(t + kb + vb + hb);
  void* st = t + kb + vb + 2u * hb;
  // 8 passes: in -> temp -> out -> temp -> ... -> out (an even number of passes ends in out)
  const uint64_t* ksrc = keys_in;
  const uint32_t* vsrc = vals_in;
  for (uint32_t pass = 0; pass < 8u; ++pass) {
    uint64_t* kdst = (pass & 1u) ? keys_out : kt;
    uint32_t* vdst = (pass & 1u) ? vals_out : vt;
    const uint32_t shift = 8u * pass;
    hipLaunchKernelGGL(k_rs_hist, dim3(tiles), dim3(kSortBlock), 0, s, ksrc, n, shift, tiles, hist);
    size_t sb = scan_bytes;
    hipError_t e = scan_u32(st, sb, hist, start, hn, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rs_scatter, dim3(tiles), dim3(kSortBlock), 0, s, ksrc, vsrc, n, shift, tiles, start, kdst, vdst);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    ksrc = kdst;
    vsrc = vdst;
  }
  return hipSuccess;
}

}  // namespace sptr
