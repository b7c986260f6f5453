// Per-table LDS radix sort of the embedding backward (tbe_bwd.hip's pipeline step 2) as a
// workgroup-size-generic body: 1024 threads x 4 items in the lookup launch / the backward
// (tbe_bwd.hip), 256 threads x 8 items as an extra role of a grouped GEMM launch (gemm.hip,
// LaunchRole phase 3: the sort needs only the indices, so it can ride on any launch before
// the update - its LDS passes are latency-bound, the GEMM tiles MFMA-bound).
#pragma once
#include "tbe_common.hpp"

namespace {

constexpr int kDigitBits = 8;
// Tables of at most this many lookups take the rank sort (n broadcast LDS keys per element,
// n^2 / 32 VALU lane-operations in all) instead of the radix passes (segsort_body).
constexpr int kRankSortMax = 512;

// TH threads x IT items per thread; PACKED: each item's local bag rides in the high bits of
// its position (pos < 2^kPosBits), so no per-position bag table is needed (the 256-thread
// role then fits in 21 KB of LDS, under the 64x32 GEMM tile's 27.6 KB).
constexpr int kPosBits = 11;
template <int TH, int IT, bool PACKED>
struct alignas(16) SegLds {
  static constexpr int kCap = TH * IT, kWaves = TH / 64;
  uint32_t key[kCap];
  int32_t pos[kCap];
  uint32_t cnt[(1 << kDigitBits) * (kWaves + 1)];  // per (digit, wave): count, then offset
  uint32_t wsum[kWaves];
  int32_t bag[PACKED ? 1 : kCap];  // bag of each local position (unpacked form)
};

// Stable LSD radix sort of TH*IT (key, pos) pairs, 8-bit digits.  Items sit in a
// wave-striped arrangement: item u of lane l in wave w is element w*64*IT + u*64 + l.  A
// digit's rank inside a wave comes from ballots (lanes holding the same digit, those below
// this lane) plus the wave's running count of that digit in LDS; one scan over the
// (digit, wave) counts gives every element its destination.  Order inside a digit is
// (wave, item, lane) = element order: stable.
template <int TH, int IT, bool PACKED>
__device__ __forceinline__ void seg_radix_sort(uint32_t (&key)[IT], int32_t (&pos)[IT], int bits,
                                               SegLds<TH, IT, PACKED>& sm) {
  constexpr int W = TH / 64;
  constexpr int NB = 1 << kDigitBits;
  constexpr int NC = NB * W;
  constexpr int CPT = NC / TH;  // counters per thread in the scan
  constexpr int CS = W + 1;     // counter row stride: digits of one wave's lanes land in
                                // distinct LDS banks
  static_assert(W % CPT == 0, "scan entries of one thread share a digit");
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const uint64_t below = (1ull << l) - 1;
  for (int s = 0; s < bits; s += kDigitBits) {
    for (int i = tid; i < NB * CS; i += TH) sm.cnt[i] = 0;
    __syncthreads();
    uint32_t rank[IT];
    uint32_t dig[IT];
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const uint32_t d = (key[u] >> s) & (NB - 1);
      uint64_t peers = ~0ull;
#pragma unroll
      for (int b = 0; b < kDigitBits; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1);
        peers &= ((d >> b) & 1) ? bal : ~bal;
      }
      const uint32_t r = __popcll(peers & below);
      const uint32_t c = __popcll(peers);
      const uint32_t base = sm.cnt[d * CS + w];
      rank[u] = base + r;
      dig[u] = d;
      if (r == c - 1) sm.cnt[d * CS + w] = base + c;  // last peer publishes
    }
    __syncthreads();
    // exclusive scan of cnt in (digit, wave) order
    uint32_t v[CPT];
    uint32_t tsum = 0;
    // logical entries tid*CPT .. +CPT-1 = digit jd, waves jw .. jw+CPT-1
    const int jd = (tid * CPT) / W, jw = (tid * CPT) % W;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      v[k] = sm.cnt[jd * CS + jw + k];
      tsum += v[k];
    }
    uint32_t inc = tsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (l >= o) inc += y;
    }
    if (l == 63) sm.wsum[w] = inc;
    __syncthreads();
    uint32_t run = inc - tsum;
    // waves before this one: all wave totals read at once (independent LDS reads)
#pragma unroll
    for (int k = 0; k < W; ++k) run += k < w ? sm.wsum[k] : 0u;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      sm.cnt[jd * CS + jw + k] = run;
      run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const uint32_t dst = sm.cnt[dig[u] * CS + w] + rank[u];
      sm.key[dst] = key[u];
      sm.pos[dst] = pos[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int e = w * (IT * 64) + u * 64 + l;
      key[u] = sm.key[e];
      pos[u] = sm.pos[e];
    }
    __syncthreads();
  }
}

// Workgroup t < T: table t's local row keys (out-of-range rows -> rows_t, DLRM_TBE_ERR_INDEX),
// stable-sorted by (row, position) over bit_width(rows_t) bits, written as global rows /
// positions / bags into the table's own range of the output.  Workgroup T marks the lookups
// outside all bags (before off[0] / after off[T*B]) as sentinels.  A table with more than
// TH*IT lookups (the caller's bound was an underestimate) is not sorted: its lookups become
// sentinels and DLRM_TBE_ERR_TABLE_CAP is raised.  Bitwise the same output for any TH x IT.
template <int TH, int IT, bool PACKED, typename IdxT, typename OffT>
__device__ __forceinline__ void segsort_body(
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const int64_t* __restrict__ row_base,
    int T, int B, int64_t N, uint32_t sentinel, uint32_t* __restrict__ keys_out,
    int32_t* __restrict__ pos_out, int32_t* __restrict__ bag_of, int32_t* __restrict__ err, int t,
    SegLds<TH, IT, PACKED>& sm) {
  constexpr int kCap = TH * IT;
  static_assert(!PACKED || kCap <= (1 << kPosBits), "packed positions");
  const int tid = threadIdx.x;
  if (t == T) {  // lookups outside every bag
    const int64_t a = (int64_t)off[0], e = (int64_t)off[(int64_t)T * B];
    for (int64_t p = tid; p < N; p += TH) {
      if (p >= a && p < e) continue;
      keys_out[p] = sentinel;
      pos_out[p] = (int32_t)p;
      bag_of[p] = -1;
    }
    return;
  }
  const int64_t s0 = (int64_t)off[(int64_t)t * B];
  const int64_t n64 = (int64_t)off[(int64_t)(t + 1) * B] - s0;  // <= kCap (contract)
  const int64_t rb = row_base[t];
  const int64_t nrows = row_base[t + 1] - rb;
  if (n64 > kCap) {  // contract violated: skip the table, report
    for (int b = tid; b < B; b += TH) {
      const int64_t a = (int64_t)off[(int64_t)t * B + b], e = (int64_t)off[(int64_t)t * B + b + 1];
      for (int64_t p = a; p < e; ++p) bag_of[p] = t * B + b;
    }
    for (int64_t i = tid; i < n64; i += TH) {
      keys_out[s0 + i] = sentinel;
      pos_out[s0 + i] = (int32_t)(s0 + i);
    }
    if (tid == 0 && err) atomicOr(err, DLRM_TBE_ERR_TABLE_CAP);
    return;
  }
  const int n = (int)n64;
  int bits = 1;
  while (bits < 32 && ((int64_t)1 << bits) <= nrows) ++bits;  // keys in [0, nrows]
  const uint32_t pad = bits >= 32 ? 0xffffffffu : (uint32_t)(((uint64_t)1 << bits) - 1);
  const int w = tid >> 6, l = tid & 63;
  // all global loads of the table are issued before the first one is consumed (one
  // memory latency, not one per loop trip): the lookup rows, then the bag offsets
  IdxT rv[IT];
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = w * (IT * 64) + u * 64 + l;  // wave-striped element order
    rv[u] = i < n ? idx[s0 + i] : (IdxT)0;
  }
  // bag of each local position, in LDS (PACKED: table-local bag, in the position array,
  // folded into each item's position below); written out in SORTED order (bag_of[i] =
  // bag of the i-th sorted lookup), which spares the block kernel a dependent load
  int32_t* bags = PACKED ? sm.pos : sm.bag;
  const OffT* toff = off + (int64_t)t * B;
  constexpr int kBU = 4;  // bags per thread per round, loads in flight
  for (int b0 = 0; b0 < B; b0 += kBU * TH) {
    int64_t ba[kBU], be[kBU];
#pragma unroll
    for (int k = 0; k < kBU; ++k) {
      const int b = b0 + k * TH + tid;
      ba[k] = b < B ? (int64_t)toff[b] : 0;
      be[k] = b < B ? (int64_t)toff[b + 1] : 0;
    }
#pragma unroll
    for (int k = 0; k < kBU; ++k) {
      const int32_t bag = (PACKED ? 0 : t * B) + b0 + k * TH + tid;
      for (int64_t p = ba[k]; p < be[k]; ++p) bags[p - s0] = bag;
    }
  }
  __syncthreads();  // bags complete
  uint32_t key[IT];
  int32_t pos[IT];
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = w * (IT * 64) + u * 64 + l;
    key[u] = pad;
    pos[u] = i;
    if (i < n) {
      const int64_t r = (int64_t)rv[u];
      key[u] = (r >= 0 && r < nrows) ? (uint32_t)r : (uint32_t)nrows;
      if (key[u] == (uint32_t)nrows && err) atomicOr(err, DLRM_TBE_ERR_INDEX);
      if constexpr (PACKED) pos[u] = i | (bags[i] << kPosBits);
    }
  }
  if (n <= TH && n <= kRankSortMax) {
    // Short tables (small batches: <= 512 lookups per table): a stable rank sort instead of
    // bits / 8 radix passes of five barriers each.  Element i's destination is
    // #{j : key_j < key_i or (key_j == key_i and j < i)} - the (key, element) order the
    // stable radix sort produces, so the output is bitwise the radix path's.  One element
    // per thread; every lane walks the same LDS keys (broadcast reads): before its wave's
    // own elements j < i for every lane (count key_j <= k), after them j > i (key_j < k),
    // the 64 in between per element - two VALU operations per key outside the diagonal.
    __syncthreads();  // (PACKED: bags in sm.pos were read above; sm.key is free)
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const int i = w * (IT * 64) + u * 64 + l;
      if (i < n) {
        sm.key[i] = key[u];
        if constexpr (PACKED) sm.pos[i] = pos[u];  // pos[u] = i | (bag << kPosBits)
      }
    }
    if (tid < 4) sm.key[n + tid] = 0xffffffffu;  // pad: never < a key (keys <= nrows)
    __syncthreads();
    if (tid < n) {
      const uint32_t k = sm.key[tid];
      const int wb = tid & ~63, we = wb + 64 < n ? wb + 64 : n;
      uint32_t rank = 0;
      for (int j = 0; j < wb; j += 4) {
        const uint4 q = *reinterpret_cast<const uint4*>(sm.key + j);
        rank += (q.x <= k) + (q.y <= k) + (q.z <= k) + (q.w <= k);
      }
      for (int j = wb; j < we; ++j) {
        const uint32_t q = sm.key[j];
        rank += (q < k) | ((q == k) & (j < tid));
      }
      for (int j = we; j < n; j += 4) {
        const uint4 q = *reinterpret_cast<const uint4*>(sm.key + j);
        rank += (q.x < k) + (q.y < k) + (q.z < k) + (q.w < k);
      }
      keys_out[s0 + rank] = k < (uint32_t)nrows ? (uint32_t)(rb + k) : sentinel;
      pos_out[s0 + rank] = (int32_t)(s0 + tid);
      if constexpr (PACKED)
        bag_of[s0 + rank] = t * B + (sm.pos[tid] >> kPosBits);
      else
        bag_of[s0 + rank] = sm.bag[tid];
    }
    return;
  }
  // (PACKED: the sort's first scatter into sm.pos comes after three barriers)
  seg_radix_sort<TH, IT, PACKED>(key, pos, bits, sm);
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int i = w * (IT * 64) + u * 64 + l;
    if (i < n) {
      keys_out[s0 + i] = key[u] < (uint32_t)nrows ? (uint32_t)(rb + key[u]) : sentinel;
      if constexpr (PACKED) {
        pos_out[s0 + i] = (int32_t)(s0 + (pos[u] & ((1 << kPosBits) - 1)));
        bag_of[s0 + i] = t * B + (pos[u] >> kPosBits);
      } else {
        pos_out[s0 + i] = (int32_t)(s0 + pos[u]);
        bag_of[s0 + i] = sm.bag[pos[u]];
      }
    }
  }
}

}  // namespace
