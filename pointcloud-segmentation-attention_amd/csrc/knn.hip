// k-nearest-neighbour grouping for gfx950: knn_point and select_top_k.
//
// Replaces SelectionSortGpuOp / selection_sort_gpu (tf_grouping.cpp:108-137,
// tf_grouping_g.cu:83-123) and the TF graph of knn_point (tf_grouping.py:48-73: a tiled
// (b,m,n,c) difference tensor, reduce_sum of squares, then select_top_k), which the reference
// runs as one GPU thread per query doing a k-step selection sort over a materialised n-long
// row. Exact semantics kept: the reference's partial selection sort moves the element at
// position s to the minimum's position at every step, so among EQUAL values the output order
// is the result of those swaps, not index order (tf_grouping_g.cu:104-120). Reproduced by
// simulating exactly those swaps on the only elements that can matter.
//
// Design: one wavefront per query row.
//  1. radix select (4 passes of 8 bits, LDS histogram per wave) finds v_k, the k-th smallest
//     value (float bits mapped to an order-preserving uint32);
//  2. a compaction pass collects the candidates: every value < v_k, every value == v_k at a
//     position < k, and the first k values == v_k at positions >= k (at most 3k entries).
//     Elements at positions >= k move only when chosen, and at most k are chosen, so no
//     other element can be selected or displaced in a way that matters;
//  3. the k selection-sort steps run on the candidate list: the minimum by (value, current
//     position) is chosen, the candidate at position s (if any) moves to the chosen one's
//     position. Step s also records that position (p_s) so that the full permuted rows of
//     select_top_k can be rebuilt as the original row with k transpositions applied.
// Distances for knn_point are recomputed in each pass (c channels summed left to right),
// never materialised: the (b,m,n) matrix of the reference is 128 MiB at SA1 sizes.
#include "common.h"

namespace pn2 {
namespace {

constexpr int kBlock = 256;
constexpr int kRowsPerBlock = kBlock / kWave;

PN2_DEV uint32_t order_key(float v) {  // ascending uint32 <=> ascending float (no NaN)
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
PN2_DEV float key_value(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

PN2_DEV int wave_scan_incl(int v, int lane) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int u = __shfl_up(v, o, kWave);
    if (lane >= o) v += u;
  }
  return v;
}

struct Cand {
  uint32_t key;
  int pos;   // current position in the row being selection-sorted
  int orig;  // index in the input row
};

// XYZ: values are squared distances from query j to the n points of cloud b (knn_point);
// otherwise rows of the given (b,m,n) matrix (select_top_k).
template <bool XYZ>
__global__ __launch_bounds__(kBlock) void knn_select_kernel(
    const float* __restrict__ xyz1, const float* __restrict__ xyz2, int c,
    const float* __restrict__ dist, int n, int m, int rows, int k, float* __restrict__ topv,
    int32_t* __restrict__ topi, int32_t* __restrict__ swap_pos) {
  __shared__ uint32_t hist[kRowsPerBlock][256];
  extern __shared__ Cand cand_all[];  // kRowsPerBlock x 3k
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int row = blockIdx.x * kRowsPerBlock + w;
  if (row >= rows) return;  // no barriers in this kernel
  Cand* cand = cand_all + (size_t)w * 3 * k;
  uint32_t* H = hist[w];
  const int b = row / m;
  const float* __restrict__ P = XYZ ? xyz1 + (size_t)b * n * c : nullptr;
  const float* __restrict__ Qr = XYZ ? xyz2 + (size_t)row * c : nullptr;
  const float* __restrict__ D = XYZ ? nullptr : dist + (size_t)row * n;
  auto key_of = [&](int t) -> uint32_t {
    if constexpr (XYZ) {
      const float* x = P + (size_t)t * c;
      float e = x[0] - Qr[0];
      float acc = e * e;
      for (int a = 1; a < c; ++a) {
        e = x[a] - Qr[a];
        acc = acc + e * e;
      }
      return order_key(acc);
    } else {
      return order_key(D[t]);
    }
  };

  // 1. radix select of the k-th smallest key (rank k-1)
  uint32_t prefix = 0, pmask = 0;
  int rank = k - 1;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = lane; i < 256; i += kWave) H[i] = 0u;
    for (int t = lane; t < n; t += kWave) {
      const uint32_t u = key_of(t);
      if ((u & pmask) == prefix) atomicAdd(&H[(u >> shift) & 255u], 1u);
    }
    const uint32_t h0 = H[4 * lane], h1 = H[4 * lane + 1], h2 = H[4 * lane + 2],
                   h3 = H[4 * lane + 3];
    const int local = (int)(h0 + h1 + h2 + h3);
    const int incl = wave_scan_incl(local, lane);
    const int excl = incl - local;
    const uint64_t mine = __ballot(excl <= rank && rank < incl);
    const int L = __ffsll((unsigned long long)mine) - 1;
    int bin = 0, before = excl;
    {
      const uint32_t hs[4] = {h0, h1, h2, h3};
      int acc = excl;
      bin = 4 * lane + 3;
      for (int q = 0; q < 4; ++q) {
        if (rank < acc + (int)hs[q]) { bin = 4 * lane + q; before = acc; break; }
        acc += (int)hs[q];
      }
    }
    bin = __shfl(bin, L, kWave);
    before = __shfl(before, L, kWave);
    prefix |= (uint32_t)bin << shift;
    pmask |= 0xFFu << shift;
    rank -= before;
  }
  const uint32_t vk = prefix;

  // 2. candidates, in position order
  const uint64_t lower = lane == 0 ? 0ull : (~0ull >> (kWave - lane));
  int nc = 0, eq_hi = 0;
  for (int base = 0; base < n; base += kWave) {
    const int t = base + lane;
    const uint32_t u = t < n ? key_of(t) : 0xFFFFFFFFu;
    const bool eqhi = t < n && u == vk && t >= k;
    const uint64_t meq = __ballot(eqhi);
    const int req = eq_hi + __popcll(meq & lower);
    const bool take = t < n && (u < vk || (u == vk && t < k) || (eqhi && req < k));
    eq_hi += __popcll(meq);
    const uint64_t mt = __ballot(take);
    if (take) {
      Cand e;
      e.key = u;
      e.pos = t;
      e.orig = t;
      cand[nc + __popcll(mt & lower)] = e;
    }
    nc += __popcll(mt);
  }

  // 3. the k selection-sort steps on the candidates (pos = -1 once chosen)
  float* V = topv + (size_t)row * k;
  int32_t* I = topi + (size_t)row * k;
  int32_t* S = swap_pos ? swap_pos + (size_t)row * k : nullptr;
  for (int s = 0; s < k; ++s) {
    uint64_t best = ~0ull;  // min of (key, pos) over unchosen candidates
    for (int e = lane; e < nc; e += kWave) {
      const Cand ce = cand[e];
      if (ce.pos >= 0) {
        const uint64_t kk = ((uint64_t)ce.key << 32) | (uint32_t)ce.pos;
        best = kk < best ? kk : best;
      }
    }
    best = ~wave_max_u64(~best);
    const uint32_t bkey = (uint32_t)(best >> 32);
    const int bpos = (int)(uint32_t)best;
    int borig = -1;
    for (int e = lane; e < nc; e += kWave) {
      Cand ce = cand[e];
      if (ce.pos == bpos) {  // the chosen one goes to position s
        borig = ce.orig;
        ce.pos = -1;
        cand[e] = ce;
      } else if (ce.pos == s) {  // the one at position s goes where the chosen one was
        ce.pos = bpos;
        cand[e] = ce;
      }
    }
    const uint64_t who = __ballot(borig >= 0);
    borig = __shfl(borig, __ffsll((unsigned long long)who) - 1, kWave);
    if (lane == 0) {
      V[s] = key_value(bkey);
      I[s] = borig;
      if (S) S[s] = bpos;
    }
  }
}

// select_top_k's full outputs: the row with positions 0..n-1, then the k transpositions
// (s, p_s) of the selection sort applied in order (tf_grouping_g.cu:93-120).
__global__ __launch_bounds__(kBlock) void selection_rows_kernel(
    const float* __restrict__ dist, int n, int rows, int k, const int32_t* __restrict__ swap_pos,
    int32_t* __restrict__ outi, float* __restrict__ out) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  const int row = blockIdx.x * kRowsPerBlock + w;
  if (row >= rows) return;
  const float* D = dist + (size_t)row * n;
  int32_t* OI = outi + (size_t)row * n;
  float* O = out + (size_t)row * n;
  for (int t = lane; t < n; t += kWave) {
    OI[t] = t;
    O[t] = D[t];
  }
  __threadfence_block();
  if (lane == 0) {
    const int32_t* S = swap_pos + (size_t)row * k;
    for (int s = 0; s < k; ++s) {
      const int p = S[s];
      if (p != s) {
        const float tv = O[p]; O[p] = O[s]; O[s] = tv;
        const int32_t ti = OI[p]; OI[p] = OI[s]; OI[s] = ti;
      }
    }
  }
}

}  // namespace
}  // namespace pn2

extern "C" {

int pn2_knn_point(const float* xyz1, const float* xyz2, int B, int n, int m, int c, int k,
                  float* val, int32_t* idx, pn2_stream_t stream) {
  if (B < 0 || n < 0 || m < 0 || c <= 0 || k <= 0 || k > n || k > 1024) return PN2_EINVAL;
  const long long rows = (long long)B * m;
  if (rows == 0) return PN2_OK;
  if (!xyz1 || !xyz2 || !val || !idx || rows > INT32_MAX) return PN2_EINVAL;
  const size_t lds = (size_t)pn2::kRowsPerBlock * 3 * k * sizeof(pn2::Cand);
  hipLaunchKernelGGL(pn2::knn_select_kernel<true>,
                     dim3((unsigned)((rows + pn2::kRowsPerBlock - 1) / pn2::kRowsPerBlock)),
                     dim3(pn2::kBlock), lds, (hipStream_t)stream, xyz1, xyz2, c, nullptr, n, m,
                     (int)rows, k, val, idx, nullptr);
  PN2_RETURN_LAUNCH();
}

int pn2_select_top_k(const float* dist, int B, int m, int n, int k, int32_t* outi, float* out,
                     int32_t* workspace, pn2_stream_t stream) {
  if (B < 0 || n < 0 || m < 0 || k <= 0 || k > n || k > 1024) return PN2_EINVAL;
  const long long rows = (long long)B * m;
  if (rows == 0) return PN2_OK;
  if (!dist || !outi || !out || !workspace || rows > INT32_MAX) return PN2_EINVAL;
  // workspace: rows x k of top values (as float), top indices and swap positions
  float* tv = reinterpret_cast<float*>(workspace);
  int32_t* ti = workspace + rows * k;
  int32_t* sp = workspace + 2 * rows * k;
  const unsigned grid = (unsigned)((rows + pn2::kRowsPerBlock - 1) / pn2::kRowsPerBlock);
  const size_t lds = (size_t)pn2::kRowsPerBlock * 3 * k * sizeof(pn2::Cand);
  hipLaunchKernelGGL(pn2::knn_select_kernel<false>, dim3(grid), dim3(pn2::kBlock), lds,
                     (hipStream_t)stream, nullptr, nullptr, 0, dist, n, m, (int)rows, k, tv, ti,
                     sp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(pn2::selection_rows_kernel, dim3(grid), dim3(pn2::kBlock), 0,
                     (hipStream_t)stream, dist, n, (int)rows, k, sp, outi, out);
  PN2_RETURN_LAUNCH();
}

size_t pn2_select_top_k_workspace_size(int B, int m, int k) {
  if (B <= 0 || m <= 0 || k <= 0) return 0;
  return (size_t)B * m * k * 3 * sizeof(int32_t);
}

}  // extern "C"
