// Table-batched EmbeddingBag backward with the optimizer fused in — deterministic.
//
// Replaces the EmbeddingBag sparse backward + torch.optim.SGD sparse add_ of the
// reference step (dlrm_s_pytorch.py:1923-1934; exact-SGD TBE of create_emb_batched
// :321-334) and the sparse branch of RWSAdagrad.step (optim/rwsadagrad.py:92-115).
//
// Pipeline (all on the caller's stream, no host sync, graph-capturable):
//  1. keys:    per lookup l, global row row_base[t] + idx[l] (or a sentinel) and its bag;
//  2. sort:    stable LSD radix sort of (row, l) pairs on ceil(log2 rows) bits (hand-written:
//              per-table LDS sort, tiled per-table passes, or device-wide passes; below);
//  3. blocks:  the sorted lookups are cut into fixed blocks (16 lookups; 64 from 2^18
//              lookups per call, tbe_bwd_roles.hpp CH / kLongCH).  One lane-group per
//              block walks them in order (row ids / grad-row offsets loaded coalesced and
//              broadcast by wave shuffles, four gradient rows in flight), summing the
//              gradient of each run of equal rows.  A run that starts and ends inside
//              the block is applied at once (one read + one write of the weight row);
//              a run crossing a block edge leaves its partial sum in slot
//              2*block + (segment starts at the block edge ? 0 : 1) — unique because a
//              block holds at most one continuing and one starting multi-block run;
//  4. combine: the block where a multi-block run starts sums its partials in block
//              order and applies the update.
// Skewed rows (the 3- and 4-row Terabyte tables receive ~700 lookups per row per
// batch) are thus split over many lane-groups instead of serialising one of them, and
// the summation order is fixed by the sort: bitwise reproducible run to run.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "mlp_rows.hpp"
#include "tbe_bwd_roles.hpp"
#include "tbe_sort.hpp"
#include "tbe_common.hpp"

namespace {


// ---------------------------------------------------------------- backward --
// Per-lookup key: global row (row_base[t] + idx) or sentinel (out of range / outside bags),
// its position and its bag.  One wave per bag (the lanes stride over the bag's lookups:
// coalesced, no search); the workgroups past the bags cover the lookups outside every bag
// (before off[0] / from off[T*B]).  KEYS = 0 (the tiled sort takes its keys from the
// indices itself): only bag_of, plus sentinel keys / positions of the outside lookups
// written straight into the sorted arrays (keys / pos then point at keys_out / pos_out).
constexpr int kBagWaves = 4;     // bags per 256-thread workgroup
constexpr int kOutsideBlocks = 16;
// (as a device function over 256-thread virtual blocks: the tiled sort's first launch runs
// it beside its pass-0 digit counts, tbe_keys_hist_kernel)
template <typename IdxT, typename OffT, typename KeyT, bool KEYS>
__device__ __forceinline__ void keys_body(
    int64_t blk, int tid, const IdxT* __restrict__ idx, const OffT* __restrict__ off,
    const int64_t* __restrict__ row_base, int T, int B, int64_t N, KeyT sentinel,
    KeyT* __restrict__ keys, int32_t* __restrict__ pos, int32_t* __restrict__ bag_of,
    int32_t* __restrict__ err) {
  constexpr int kDim = 256;
  const int64_t nb = (int64_t)T * B;
  const int64_t bag_blocks = (nb + kBagWaves - 1) / kBagWaves;
  const int lane = tid & 63;
  if (blk >= bag_blocks) {  // lookups outside every bag
    const int64_t a = (int64_t)off[0], e = (int64_t)off[nb];
    const int64_t stride = (int64_t)kOutsideBlocks * kDim;
    const int64_t g = (blk - bag_blocks) * kDim + tid;
    auto mark = [&](int64_t p) {  // (the tiled sort keeps these: -1 reads as "no bag" too
      keys[p] = sentinel;          //  when the sorted values are bags)
      pos[p] = KEYS ? (int32_t)p : -1;
      bag_of[p] = -1;
    };
    for (int64_t p = g; p < a && p < N; p += stride) mark(p);
    for (int64_t p = e + g; p < N; p += stride) mark(p);
    return;
  }
  const int64_t bag = blk * kBagWaves + (tid >> 6);
  if (bag >= nb) return;
  const int t = (int)(bag / B);
  const int64_t a = (int64_t)off[bag], e = (int64_t)off[bag + 1];
  const int64_t rb = row_base[t], nrows = row_base[t + 1] - rb;
  for (int64_t p = a + lane; p < e; p += 64) {
    const int64_t r = (int64_t)idx[p];
    const bool ok = r >= 0 && r < nrows;
    if (!ok && err) atomicOr(err, DLRM_TBE_ERR_INDEX);
    if constexpr (KEYS) {
      keys[p] = ok ? (KeyT)(rb + r) : sentinel;
      pos[p] = (int32_t)p;
    }
    bag_of[p] = ok ? (int32_t)bag : -1;
  }
}

template <typename IdxT, typename OffT, typename KeyT, bool KEYS>
__global__ __launch_bounds__(256) void tbe_bwd_keys_kernel(
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const int64_t* __restrict__ row_base,
    int T, int B, int64_t N, KeyT sentinel, KeyT* __restrict__ keys, int32_t* __restrict__ pos,
    int32_t* __restrict__ bag_of, int32_t* __restrict__ err) {
  keys_body<IdxT, OffT, KeyT, KEYS>(blockIdx.x, threadIdx.x, idx, off, row_base, T, B, N, sentinel,
                                    keys, pos, bag_of, err);
}

inline int64_t keys_grid(int T, int B) {
  return ((int64_t)T * B + kBagWaves - 1) / kBagWaves + kOutsideBlocks;
}

// Per-table sort (replaces keys + device radix sort when every table's lookups fit in
// one workgroup): workgroup t builds table t's local row keys (out-of-range rows ->
// rows_t) and sorts (key, position) with a stable LDS radix sort over only
// bit_width(rows_t) bits, then writes global rows / positions into the table's own range
// of the output.  Stable on positions, so the order equals the device-wide stable sort.
// Tables own disjoint row ranges and consecutive lookup ranges, so the concatenation is
// a valid grouping for the block kernel.  Workgroup T marks the lookups outside all bags
// (before off[0] / after off[T*B]) as sentinels.  A table with more than kSegCap lookups
// (the caller's max_lookups_per_table was an underestimate) is not sorted: all its lookups
// become sentinels (no update, no stale keys, no out-of-bounds row) and bit
// DLRM_TBE_ERR_TABLE_CAP is raised in *err.
constexpr int kSegThreads = 1024, kSegItems = 4;
constexpr int kSegCap = kSegThreads * kSegItems;  // lookups per table
using SegSortLds = SegLds<kSegThreads, kSegItems, false>;

template <typename IdxT, typename OffT>
__global__ __launch_bounds__(kSegThreads) void tbe_bwd_segsort_kernel(
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const int64_t* __restrict__ row_base,
    int T, int B, int64_t N, uint32_t sentinel, uint32_t* __restrict__ keys_out,
    int32_t* __restrict__ pos_out, int32_t* __restrict__ bag_of, int32_t* __restrict__ err) {
  __shared__ SegSortLds sm;
  segsort_body<kSegThreads, kSegItems, false, IdxT, OffT>(idx, off, row_base, T, B, N, sentinel,
                                                          keys_out, pos_out, bag_of, err,
                                                          blockIdx.x, sm);
}

// The forward gather and the backward's per-table sort in ONE launch: the sort depends only
// on the indices, and its T+1 latency-bound workgroups (LDS radix passes on T CUs) run beside
// the bandwidth-bound gather instead of as a separate launch in the backward.  Blocks
// [0, T] sort (started first), the rest gather.  512 threads per workgroup.
// With mlp_blocks > 0 a third role, the bottom MLP forward (mlp_rows.hpp), takes blocks
// [nsort, nsort+mlp_blocks): it reads only X and the bottom weights, independent of the rest.
// nsort = T + 1 with the sort, 0 without it (tables too large for the per-table LDS sort,
// e.g. C1's L = 100: the lookup and the bottom MLP still share one launch - the gather is
// HBM-bound, the MLP rides on MFMA and LDS).
constexpr int kPreThreads = kSegThreads;
static_assert(kPreThreads == kMlpWaves * 64, "one workgroup size for every role");
union PresortLds {
  SegSortLds sort;
  float mlp[kMlpLdsFloats];
};
template <int LPB, int VW, int MAXV, typename IdxT, typename OffT>
__global__ __launch_bounds__(kPreThreads) void tbe_fwd_presort_kernel(
    const float* __restrict__ W, int64_t D, const int64_t* __restrict__ row_base, int T, int B,
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const float* __restrict__ psw,
    float* __restrict__ out, int64_t out_bs, int32_t* __restrict__ err, int64_t N,
    uint32_t sentinel, uint32_t* __restrict__ keys_out, int32_t* __restrict__ pos_out,
    int32_t* __restrict__ bag_of, const MlpChain mc, int mlp_blocks, int nsort) {
  __shared__ __attribute__((aligned(16))) PresortLds sm;
  const int b = blockIdx.x;
  if (b < nsort) {
    segsort_body<kSegThreads, kSegItems, false, IdxT, OffT>(idx, off, row_base, T, B, N,
                                                            sentinel, keys_out, pos_out, bag_of,
                                                            err, b, sm.sort);
    return;
  }
  if (b < nsort + mlp_blocks) {
    mlp_rows_body(mc, b - nsort, sm.mlp);
    return;
  }
  const int g0 = nsort + mlp_blocks;
  tbe_fwd_body<LPB, VW, MAXV, IdxT, OffT>(W, D, row_base, T, B, idx, off, psw, out, out_bs, err,
                                          (int64_t)b - g0, (int64_t)gridDim.x - g0);
}

__global__ __launch_bounds__(kMlpWaves * 64) void mlp_chain_kernel(const MlpChain mc) {
  __shared__ __attribute__((aligned(16))) float lds[kMlpLdsFloats];
  mlp_rows_body(mc, blockIdx.x, lds);
}



// The per-table LDS sort applies (and dlrm_tbe_forward_presort can run it early).
inline bool presort_applies(size_t key_bytes, int64_t max_seg, int64_t N) {
  return key_bytes == 4 && max_seg > 0 && max_seg <= kSegCap && N < (int64_t)0x7fffffff;
}

inline int bit_width_u64(uint64_t v) {
  int b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b < 1 ? 1 : b;
}

// ------------------------------------------------ tiled per-table radix sort --
// Tables with more lookups than one workgroup sorts (kSegCap: e.g. L = 100 pooling) and
// 32-bit keys: a stable LSD radix sort of each table's (local row, position) pairs in its
// own lookup range, DB-bit digits, tiles of kTile lookups.  Per pass, three launches:
//   hist:    tile (t, j) counts its digits (LDS atomics) -> hist[t][d][j];
//   scan:    per table, exclusive scan of hist in (digit, tile) order;
//   scatter: tile (t, j) ranks its lookups by digit (wave ballots + per-(digit, wave)
//            running counts in LDS: element order kept, so stable) and writes each to
//            table start + hist[t][d][j] + its rank among the tile's digit-d lookups.
// Same (row, position) order as the device-wide sort and the per-table LDS sort; no
// memsets, no decoupled look-back.  The keys kernel has written bag_of (by lookup
// position) and the sentinels of the lookups outside every bag.  A table with more
// lookups than its J tiles cover (max_lookups_per_table underestimated) is not sorted: its
// range becomes sentinels (no update) and DLRM_TBE_ERR_TABLE_CAP is raised.
constexpr int kTileThreads = 1024, kTileItems = 4, kTile = kTileThreads * kTileItems;
constexpr int kTileWaves = kTileThreads / 64;
// the scatter pass: the same 4096-lookup tiles on 512 threads x 8 items - half the per-
// (digit, wave) counters, so two workgroups share a CU (C1 scatter 23.3 -> 18.5 us); the
// stable rank is by element index in either arrangement
constexpr int kScatThreads = 512, kScatItems = kTile / kScatThreads;
constexpr int kScatWaves = kScatThreads / 64;

struct TiledPass {
  const int64_t* row_base;
  int T, B, J;          // tables, bags per table, tiles per table
  int shift;            // digit shift of this pass
  int first, last;      // pass 0 reads the indices; the last pass writes global keys
  const uint32_t* kin;  // pass input (pass > 0)
  const int32_t* pin;
  uint32_t* kout;       // pass output
  int32_t* pout;
  uint32_t* hist;       // [T][2^DB][J]
  uint32_t sentinel;    // global sentinel key (last pass)
  int32_t* err;
  int global;           // one segment [0, n_all) of global keys read from kin/pin in pass 0
  int64_t n_all;
  const int32_t* bag_of;  // non-null: the sorted values are BAGS (bag_of[position], read
                          // coalesced in pass 0) instead of positions, so the block kernel
                          // reads each lookup's bag in sorted order (no dependent gather)
  // per-table passes (not global): a table of nrows rows needs ceil(bit_width(nrows) / DB)
  // passes, at most npass; pass ps of such a table reads / writes the (ka, pa) or the
  // final (ko, po) pair so that its own last pass lands in (ko, po), and passes past its
  // own count skip it (e.g. 1 M-row tables in an 8 M-row call: 2 passes of 10 bits, not 3)
  uint32_t* ka;
  int32_t* pa;
  uint32_t* ko;
  int32_t* po;
  int ps, npass;
  // the scan in chunks of JC tiles, C per table: csum[t][c][digit] = the chunk's counts
  uint32_t* csum;
  int C, JC;
  // wide scan (tiles per table <= kWideScanMaxJ): hist[t][j][d] becomes the count of digit
  // d in the table's tiles before j, csum[t][0][d] the digit's total; the scatter adds the
  // digit's start (the exclusive scan of the totals) itself
  int wide;
};

// The pass as table t sees it (global mode: the host's ping-pong as given).
struct PassView {
  bool skip, first, last;
  const uint32_t* kin;
  const int32_t* pin;
  uint32_t* kout;
  int32_t* pout;
  int shift;      // this pass's digit: (key >> shift) & mask
  uint32_t mask;
};

template <int DB>
__device__ __forceinline__ PassView pass_view(const TiledPass& a, int64_t nrows) {
  PassView v{};
  if (a.global) {
    v.first = a.first, v.last = a.last, v.kin = a.kin, v.pin = a.pin;
    v.kout = a.kout, v.pout = a.pout;
    v.shift = a.shift, v.mask = (1u << DB) - 1;
    return v;
  }
  int bits = 1;
  while (bits < 32 && ((int64_t)1 << bits) <= nrows) ++bits;  // keys in [0, nrows]
  int passes = (bits + DB - 1) / DB;
  if (passes > a.npass) passes = a.npass;
  // the table's bits split evenly over its passes (17 bits: 9 + 8, not 10 + 7): fewer
  // digits in the first pass, so each tile's runs per digit - the scatter's store segments -
  // are longer (a stable LSD sort by any digit split gives the same order)
  const int width = (bits + passes - 1) / passes < DB ? (bits + passes - 1) / passes : DB;
  v.shift = a.ps * width;
  v.mask = (1u << width) - 1;
  v.skip = a.ps >= passes;
  v.first = a.ps == 0;
  v.last = a.ps == passes - 1;
  const bool out_final = ((passes - 1 - a.ps) & 1) == 0;
  const bool in_final = ((passes - a.ps) & 1) == 0;
  v.kout = out_final ? a.ko : a.ka;
  v.pout = out_final ? a.po : a.pa;
  v.kin = a.ps == 0 ? nullptr : (in_final ? a.ko : a.ka);
  v.pin = a.ps == 0 ? nullptr : (in_final ? a.po : a.pa);
  return v;
}

template <int DB>
struct TiledLds {
  uint32_t cnt[(1 << DB) * (kScatWaves + 1)];  // per (digit, wave)
  uint32_t dstart[1 << DB];                     // tile-local start of each digit
  uint32_t wsum[kScatWaves];
  uint32_t dbase[1 << DB];                      // wide scan: the digit's start in the table
  uint32_t key[kTile];                          // the tile in digit order
  int32_t pos[kTile];
};

// Element e of tile j of table t: wave-striped (e = w*64*IT + u*64 + l), position
// s + j*kTile + e.  Loads this thread's IT (key, pos, valid).
template <int IT, typename IdxT, bool WITH_POS = true>
__device__ __forceinline__ void tiled_load(const TiledPass& a, const PassView& v,
                                           const IdxT* __restrict__ idx, int64_t s, int64_t n,
                                           int j, int64_t nrows, uint32_t (&key)[IT],
                                           int32_t (&pos)[IT], bool (&ok)[IT]) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
#pragma unroll
  for (int u = 0; u < IT; ++u) {
    const int64_t e = (int64_t)j * kTile + w * (IT * 64) + u * 64 + l;
    ok[u] = e < n;
    const int64_t p = s + (ok[u] ? e : 0);
    if (v.first && !a.global) {
      const int64_t r = (int64_t)idx[p];
      key[u] = (r >= 0 && r < nrows) ? (uint32_t)r : (uint32_t)nrows;
      if (WITH_POS) pos[u] = a.bag_of ? a.bag_of[p] : (int32_t)p;
    } else {
      key[u] = v.kin[p];
      if (WITH_POS)  // (global pass 0: pin[p] = p)
        pos[u] = (v.first && a.bag_of) ? a.bag_of[p] : v.pin[p];
    }
  }
}

template <typename OffT>
__device__ __forceinline__ bool tiled_range(const TiledPass& a, const OffT* __restrict__ off, int t,
                                            int64_t& s, int64_t& n) {
  if (a.global) {
    s = 0;
    n = a.n_all;
    return n <= (int64_t)a.J * kTile;
  }
  s = (int64_t)off[(int64_t)t * a.B];
  n = (int64_t)off[(int64_t)(t + 1) * a.B] - s;
  return n <= (int64_t)a.J * kTile;  // false: the table overflows its tiles
}

template <typename IdxT, typename OffT, int DB>
__device__ __forceinline__ void hist_body(const IdxT* __restrict__ idx,
                                          const OffT* __restrict__ off, const TiledPass& a,
                                          int blk, uint32_t* cnt) {
  constexpr int NB = 1 << DB;
  const int t = blk / a.J, j = blk - (blk / a.J) * a.J;
  int64_t s, n;
  const int64_t nrows = a.row_base[t + 1] - a.row_base[t];
  const PassView v = pass_view<DB>(a, nrows);
  if (v.skip) return;
  if (!tiled_range(a, off, t, s, n)) {
    if (v.first && j == 0 && threadIdx.x == 0 && a.err) atomicOr(a.err, DLRM_TBE_ERR_TABLE_CAP);
    return;
  }
  for (int d = threadIdx.x; d < NB; d += kTileThreads) cnt[d] = 0;
  uint32_t key[kTileItems];
  int32_t pos[kTileItems];
  bool ok[kTileItems];
  tiled_load<kTileItems, IdxT, false>(a, v, idx, s, n, j, nrows, key, pos, ok);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kTileItems; ++u)
    if (ok[u]) atomicAdd(&cnt[(key[u] >> v.shift) & v.mask], 1u);
  __syncthreads();
  uint32_t* h = a.hist + ((int64_t)t * a.J + j) * NB;
  for (int d = threadIdx.x; d < NB; d += kTileThreads) h[d] = cnt[d];
}

template <typename IdxT, typename OffT, int DB>
__global__ __launch_bounds__(kTileThreads) void tbe_tiled_hist_kernel(
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const TiledPass a) {
  __shared__ uint32_t cnt[1 << DB];
  hist_body<IdxT, OffT, DB>(idx, off, a, blockIdx.x, cnt);
}

// The tiled sort's first launch: pass 0's digit counts (workgroups [0, T J): they read only
// the indices) beside the bag-parallel keys pass (the rest, four 256-thread keys blocks per
// workgroup: bag_of and the outside-bag sentinels, read first by pass 0's scatter).
struct KeysArgs {
  const int64_t* row_base;
  int T, B;
  int64_t N;
  uint32_t sentinel;
  uint32_t* keys;
  int32_t* pos;
  int32_t* bag_of;
  int32_t* err;
  int64_t blocks;  // 256-thread keys blocks (keys_grid)
};

template <typename IdxT, typename OffT, int DB>
__global__ __launch_bounds__(kTileThreads) void tbe_keys_hist_kernel(
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const TiledPass a,
    const KeysArgs k) {
  __shared__ uint32_t cnt[1 << DB];
  const int nh = a.T * a.J;
  if ((int)blockIdx.x < nh) {
    hist_body<IdxT, OffT, DB>(idx, off, a, blockIdx.x, cnt);
    return;
  }
  const int64_t vb = ((int64_t)blockIdx.x - nh) * (kTileThreads / 256) + (threadIdx.x >> 8);
  if (vb < k.blocks)
    keys_body<IdxT, OffT, uint32_t, false>(vb, threadIdx.x & 255, idx, off, k.row_base, k.T, k.B,
                                           k.N, k.sentinel, k.keys, k.pos, k.bag_of, k.err);
}

// The exclusive scan of a table's NB * J counts in (digit, tile) order, in two launches
// over chunks of JC tiles (a table of C chunks gets C workgroups in each: the device-wide
// sort's one segment of J = N / 4096 tiles no longer walks in one workgroup - C1 shape
// 2 x 51 -> ~2 x 5 us).  hist is [t][j][d]; a thread owns DPT digits.
//   csum: workgroup (t, c) sums each digit over its chunk's tiles -> csum[t][c][d];
//   scan: workgroup (t, c) adds up the chunk sums (all chunks: the digit totals, scanned
//         across the workgroup; chunks < c: this chunk's start) and rewrites its tiles'
//         counts as base + running count.
constexpr int kScanChunk = 16, kMaxScanChunks = 64;
// One chunk (the scan walks the tiles itself, no csum launch) up to kScanOneChunk tiles
// per table: the per-table sort's tables (C1: 50 tiles) keep one launch of T workgroups.
constexpr int kScanOneChunk = 64;
inline void plan_scan_chunks(TiledPass& a) {
  a.JC = (a.J + kMaxScanChunks - 1) / kMaxScanChunks;
  if (a.JC < kScanChunk) a.JC = kScanChunk;
  if (a.J <= kScanOneChunk) a.JC = a.J > 0 ? a.J : 1;
  a.C = (a.J + a.JC - 1) / a.JC;
}

template <int DB>
__global__ __launch_bounds__(kTileThreads) void tbe_tiled_csum_kernel(const TiledPass a,
                                                                      const void* off_v,
                                                                      int off_bits) {
  constexpr int NB = 1 << DB;
  constexpr int DPT = NB / kTileThreads > 0 ? NB / kTileThreads : 1;  // digits per thread
  const int t = blockIdx.x / a.C, c = blockIdx.x - (blockIdx.x / a.C) * a.C;
  const int tid = threadIdx.x;
  int64_t s, n;
  const PassView v = pass_view<DB>(a, a.row_base[t + 1] - a.row_base[t]);
  if (v.skip) return;
  const bool fits = off_bits == 32
                        ? tiled_range(a, static_cast<const int32_t*>(off_v), t, s, n)
                        : tiled_range(a, static_cast<const int64_t*>(off_v), t, s, n);
  const int d0 = tid * DPT;
  if (!fits || d0 >= NB) return;
  const uint32_t* h = a.hist + (int64_t)t * a.J * NB;
  const int j0 = c * a.JC, j1 = j0 + a.JC < a.J ? j0 + a.JC : a.J;
  constexpr int U = 32 / DPT;
  uint32_t tot[DPT];
#pragma unroll
  for (int q = 0; q < DPT; ++q) tot[q] = 0;
  for (int jj = j0; jj < j1; jj += U) {
    uint32_t x[U][DPT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < DPT; ++q)
        x[u][q] = (jj + u < j1) ? h[(int64_t)(jj + u) * NB + d0 + q] : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < DPT; ++q) tot[q] += x[u][q];
  }
#pragma unroll
  for (int q = 0; q < DPT; ++q) a.csum[((int64_t)t * a.C + c) * NB + d0 + q] = tot[q];
}

template <int DB>
__global__ __launch_bounds__(kTileThreads) void tbe_tiled_scan_kernel(const TiledPass a,
                                                                      const void* off_v,
                                                                      int off_bits) {
  constexpr int NB = 1 << DB;
  constexpr int DPT = NB / kTileThreads > 0 ? NB / kTileThreads : 1;  // digits per thread
  static_assert(NB % kTileThreads == 0 || kTileThreads % NB == 0, "digit map");
  __shared__ uint32_t wsum[kTileWaves];
  const int t = blockIdx.x / a.C, c = blockIdx.x - (blockIdx.x / a.C) * a.C;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  int64_t s, n;
  const PassView v = pass_view<DB>(a, a.row_base[t + 1] - a.row_base[t]);
  if (v.skip) return;
  const bool fits = off_bits == 32
                        ? tiled_range(a, static_cast<const int32_t*>(off_v), t, s, n)
                        : tiled_range(a, static_cast<const int64_t*>(off_v), t, s, n);
  if (!fits) {
    if (v.last && c == 0)  // the table's range holds sentinels (no update)
      for (int64_t i = tid; i < n; i += kTileThreads) {
        v.kout[s + i] = a.sentinel;
        v.pout[s + i] = (int32_t)(s + i);
      }
    return;
  }
  uint32_t* h = a.hist + (int64_t)t * a.J * NB;
  const int j0 = c * a.JC, j1 = j0 + a.JC < a.J ? j0 + a.JC : a.J;
  constexpr int U = 32 / DPT;
  // digits d0 .. d0+DPT-1 of this thread (NB < threads: the first NB threads only)
  const int d0 = tid * DPT;
  const bool active = d0 < NB;
  uint32_t tot[DPT], pre[DPT];
#pragma unroll
  for (int q = 0; q < DPT; ++q) tot[q] = pre[q] = 0;
  if (active && a.C == 1) {  // one chunk: the digit totals straight from the tiles
    for (int jj = j0; jj < j1; jj += U) {
      uint32_t x[U][DPT];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < DPT; ++q)
          x[u][q] = (jj + u < j1) ? h[(int64_t)(jj + u) * NB + d0 + q] : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < DPT; ++q) tot[q] += x[u][q];
    }
  } else if (active) {
    const uint32_t* cs = a.csum + (int64_t)t * a.C * NB;
    for (int c0 = 0; c0 < a.C; c0 += U) {
      uint32_t x[U][DPT];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < DPT; ++q)
          x[u][q] = (c0 + u < a.C) ? cs[(int64_t)(c0 + u) * NB + d0 + q] : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < DPT; ++q) {
          tot[q] += x[u][q];
          if (c0 + u < c) pre[q] += x[u][q];
        }
    }
  }
  uint32_t tsum = 0;
#pragma unroll
  for (int q = 0; q < DPT; ++q) tsum += tot[q];
  uint32_t inc = tsum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (l >= o) inc += y;
  }
  if (l == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = inc - tsum;
#pragma unroll
  for (int k = 0; k < kTileWaves; ++k) base += k < w ? wsum[k] : 0u;
  if (!active) return;
  uint32_t run[DPT];
#pragma unroll
  for (int q = 0; q < DPT; ++q) {
    run[q] = base + pre[q];
    base += tot[q];
  }
  for (int jj = j0; jj < j1; jj += U) {
    uint32_t x[U][DPT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < DPT; ++q)
        x[u][q] = (jj + u < j1) ? h[(int64_t)(jj + u) * NB + d0 + q] : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < DPT; ++q)
        if (jj + u < j1) {
          h[(int64_t)(jj + u) * NB + d0 + q] = run[q];
          run[q] += x[u][q];
        }
  }
}

// Wide scan: workgroup (t, g) takes digits [64 g, 64 g + 64) of table t - a lane per digit,
// wave w the tiles [w JW, (w + 1) JW) - and rewrites each (tile, digit) count as the digit's
// count over the earlier tiles; the digit totals go to csum[t][0][d].  T * 2^DB / 64
// workgroups, each one round of loads (the one-chunk scan: T workgroups walking all J
// tiles of all digits, C1 11.3 us).
constexpr int kWideScanMaxJ = 2048;
template <int DB>
__global__ __launch_bounds__(kTileThreads) void tbe_tiled_wide_scan_kernel(const TiledPass a,
                                                                           const void* off_v,
                                                                           int off_bits) {
  constexpr int NB = 1 << DB, G = NB / 64;
  __shared__ uint32_t ws[kTileWaves][64];
  const int t = blockIdx.x / G, g = blockIdx.x - (blockIdx.x / G) * G;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  int64_t s, n;
  const PassView v = pass_view<DB>(a, a.row_base[t + 1] - a.row_base[t]);
  if (v.skip) return;
  const bool fits = off_bits == 32
                        ? tiled_range(a, static_cast<const int32_t*>(off_v), t, s, n)
                        : tiled_range(a, static_cast<const int64_t*>(off_v), t, s, n);
  if (!fits) {
    if (v.last && g == 0)  // the table's range holds sentinels (no update)
      for (int64_t i = tid; i < n; i += kTileThreads) {
        v.kout[s + i] = a.sentinel;
        v.pout[s + i] = (int32_t)(s + i);
      }
    return;
  }
  const int d = g * 64 + l;
  uint32_t* h = a.hist + (int64_t)t * a.J * NB + d;
  const int JW = (a.J + kTileWaves - 1) / kTileWaves;
  const int j0 = w * JW, j1 = j0 + JW < a.J ? j0 + JW : a.J;
  constexpr int U = 8;
  uint32_t sum = 0;
  for (int jj = j0; jj < j1; jj += U) {
    uint32_t x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = jj + u < j1 ? h[(int64_t)(jj + u) * NB] : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u) sum += x[u];
  }
  ws[w][l] = sum;
  __syncthreads();
  uint32_t run = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kTileWaves; ++k) {
    const uint32_t y = ws[k][l];
    run += k < w ? y : 0u;
    tot += y;
  }
  for (int jj = j0; jj < j1; jj += U) {
    uint32_t x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = jj + u < j1 ? h[(int64_t)(jj + u) * NB] : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (jj + u < j1) {
        h[(int64_t)(jj + u) * NB] = run;
        run += x[u];
      }
  }
  if (w == 0) a.csum[(int64_t)t * NB + d] = tot;
}

template <typename IdxT, typename OffT, int DB>
__global__ __launch_bounds__(kScatThreads) void tbe_tiled_scatter_kernel(
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const TiledPass a) {
  constexpr int NB = 1 << DB;
  constexpr int CS = kScatWaves + 1;  // counter row stride
  __shared__ TiledLds<DB> sm;
  const int t = blockIdx.x / a.J, j = blockIdx.x - (blockIdx.x / a.J) * a.J;
  int64_t s, n;
  const int64_t rb = a.row_base[t];
  const int64_t nrows = a.row_base[t + 1] - rb;
  const PassView v = pass_view<DB>(a, nrows);
  if (v.skip) return;
  if (!tiled_range(a, off, t, s, n)) return;
  if ((int64_t)j * kTile >= n) return;  // empty tile (uniform)
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  uint32_t key[kScatItems];
  int32_t pos[kScatItems];
  bool ok[kScatItems];
  tiled_load<kScatItems>(a, v, idx, s, n, j, nrows, key, pos, ok);
  for (int i = tid; i < NB * CS; i += kScatThreads) sm.cnt[i] = 0;
  __syncthreads();
  const uint64_t below = (1ull << l) - 1;
  uint32_t rank[kScatItems], dig[kScatItems];
#pragma unroll
  for (int u = 0; u < kScatItems; ++u) {
    const uint32_t d = (key[u] >> v.shift) & v.mask;
    uint64_t peers = __ballot(ok[u]);
#pragma unroll
    for (int b = 0; b < DB; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bal : ~bal;
    }
    const uint32_t r = __popcll(peers & below);
    const uint32_t c = __popcll(peers);
    const uint32_t base = sm.cnt[d * CS + w];
    rank[u] = base + r;
    dig[u] = d;
    if (ok[u] && r == c - 1) sm.cnt[d * CS + w] = base + c;  // last peer publishes
  }
  __syncthreads();
  // per digit: exclusive prefix over the waves, and the digit's tile total
  constexpr int DPT = NB / kScatThreads > 0 ? NB / kScatThreads : 1;
  const int d0 = tid * DPT;
  uint32_t tot[DPT];
#pragma unroll
  for (int q = 0; q < DPT; ++q) {
    tot[q] = 0;
    if (d0 + q < NB) {
      uint32_t v[kScatWaves];
#pragma unroll
      for (int k = 0; k < kScatWaves; ++k) v[k] = sm.cnt[(d0 + q) * CS + k];
#pragma unroll
      for (int k = 0; k < kScatWaves; ++k) {
        sm.cnt[(d0 + q) * CS + k] = tot[q];
        tot[q] += v[k];
      }
    }
  }
  // tile-local digit starts: exclusive scan of the totals over the workgroup
  uint32_t tsum = 0;
#pragma unroll
  for (int q = 0; q < DPT; ++q) tsum += tot[q];
  uint32_t inc = tsum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (l >= o) inc += y;
  }
  if (l == 63) sm.wsum[w] = inc;
  __syncthreads();
  uint32_t run = inc - tsum;
#pragma unroll
  for (int k = 0; k < kScatWaves; ++k) run += k < w ? sm.wsum[k] : 0u;
#pragma unroll
  for (int q = 0; q < DPT; ++q)
    if (d0 + q < NB) {
      sm.dstart[d0 + q] = run;
      run += tot[q];
    }
  __syncthreads();
  if (a.wide) {  // the digits' starts in the table: exclusive scan of the digit totals
    const uint32_t* dt = a.csum + (int64_t)t * NB;
    uint32_t x[DPT], xs = 0;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      x[q] = d0 + q < NB ? dt[d0 + q] : 0u;
      xs += x[q];
    }
    uint32_t xi = xs;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(xi, o, 64);
      if (l >= o) xi += y;
    }
    if (l == 63) sm.wsum[w] = xi;  // (the tile-local reads of wsum are behind the barrier)
    __syncthreads();
    uint32_t xr = xi - xs;
#pragma unroll
    for (int k = 0; k < kScatWaves; ++k) xr += k < w ? sm.wsum[k] : 0u;
#pragma unroll
    for (int q = 0; q < DPT; ++q)
      if (d0 + q < NB) {
        sm.dbase[d0 + q] = xr;
        xr += x[q];
      }
    __syncthreads();
  }
  // stage the tile in digit order, then write it out: consecutive threads take
  // consecutive elements, so each digit's elements go out as one contiguous run
#pragma unroll
  for (int u = 0; u < kScatItems; ++u) {
    if (!ok[u]) continue;
    const uint32_t lp = sm.dstart[dig[u]] + sm.cnt[dig[u] * CS + w] + rank[u];
    sm.key[lp] = key[u];
    sm.pos[lp] = pos[u];
  }
  __syncthreads();
  const int nt = (int)((n - (int64_t)j * kTile) < kTile ? (n - (int64_t)j * kTile) : kTile);
  const uint32_t* h = a.hist + ((int64_t)t * a.J + j) * NB;
#pragma unroll
  for (int u = 0; u < kScatItems; ++u) {
    const int i = u * kScatThreads + tid;
    if (i >= nt) continue;
    const uint32_t k = sm.key[i];
    const uint32_t d = (k >> v.shift) & v.mask;
    const int64_t dst = s + h[d] + (a.wide ? sm.dbase[d] : 0u) + (i - sm.dstart[d]);
    if (v.last && !a.global)
      v.kout[dst] = k < (uint32_t)nrows ? (uint32_t)(rb + k) : a.sentinel;
    else
      v.kout[dst] = k;
    v.pout[dst] = sm.pos[i];
  }
}

// DB-bit digits, passes over `bits` key bits (local rows <= total_rows): 10-bit digits when
// they save a pass over 8-bit ones.
inline int tiled_digit_bits(int bits) {
  return (bits + 9) / 10 < (bits + 7) / 8 ? 10 : 8;
}

template <typename IdxT, typename OffT, int DB>
void launch_tiled_sort(const IdxT* idx, const OffT* off, const int64_t* row_base, int T, int B,
                       int J, int bits, uint32_t* k_a, int32_t* p_a, uint32_t* k_out,
                       int32_t* p_out, uint32_t* hist, uint32_t sentinel, int32_t* err,
                       int off_bits, const int32_t* bag_of, const KeysArgs& keys,
                       hipStream_t st) {
  const int npass = (bits + DB - 1) / DB;
  TiledPass a{};
  a.row_base = row_base, a.T = T, a.B = B, a.J = J, a.hist = hist, a.sentinel = sentinel;
  a.err = err;
  a.bag_of = bag_of;
  // per-table ping-pong (pass_view): each table's own last pass lands in (k_out, p_out)
  a.ka = k_a, a.pa = p_a, a.ko = k_out, a.po = p_out;
  a.npass = npass;
  plan_scan_chunks(a);
  a.csum = hist + (size_t)T * J * (1 << DB);  // after the per-tile counts
  a.wide = J <= kWideScanMaxJ && (1 << DB) % 64 == 0 && dlrm::tuning(DLRM_TUNE_TBE_SORT) != 2;
  // the keys pass rides on pass 0's count launch (tuning TBE_SORT 2: its own launch first)
  const bool merged = dlrm::tuning(DLRM_TUNE_TBE_SORT) != 2 &&
                      (int64_t)T * J + dlrm::ceil_div(keys.blocks, (int64_t)(kTileThreads / 256)) <
                          (int64_t)INT32_MAX;
  if (!merged)
    hipLaunchKernelGGL((tbe_bwd_keys_kernel<IdxT, OffT, uint32_t, false>), dim3(keys.blocks),
                       dim3(256), 0, st, idx, off, keys.row_base, keys.T, keys.B, keys.N,
                       keys.sentinel, keys.keys, keys.pos, keys.bag_of, keys.err);
  for (int ps = 0; ps < npass; ++ps) {
    a.shift = ps * DB;
    a.ps = ps;
    if (ps == 0 && merged)
      hipLaunchKernelGGL((tbe_keys_hist_kernel<IdxT, OffT, DB>),
                         dim3((unsigned)(T * J + dlrm::ceil_div(keys.blocks,
                                                                (int64_t)(kTileThreads / 256)))),
                         dim3(kTileThreads), 0, st, idx, off, a, keys);
    else
      hipLaunchKernelGGL((tbe_tiled_hist_kernel<IdxT, OffT, DB>), dim3(T * J), dim3(kTileThreads),
                         0, st, idx, off, a);
    if (a.wide)
      hipLaunchKernelGGL((tbe_tiled_wide_scan_kernel<DB>), dim3(T * ((1 << DB) / 64)),
                         dim3(kTileThreads), 0, st, a, static_cast<const void*>(off), off_bits);
    else if (a.C > 1)
      hipLaunchKernelGGL((tbe_tiled_csum_kernel<DB>), dim3(T * a.C), dim3(kTileThreads), 0, st,
                         a, static_cast<const void*>(off), off_bits);
    if (!a.wide)
      hipLaunchKernelGGL((tbe_tiled_scan_kernel<DB>), dim3(T * a.C), dim3(kTileThreads), 0, st,
                         a, static_cast<const void*>(off), off_bits);
    hipLaunchKernelGGL((tbe_tiled_scatter_kernel<IdxT, OffT, DB>), dim3(T * J),
                       dim3(kScatThreads), 0, st, idx, off, a);
  }
}

// The device-wide sort (no max_lookups_per_table bound): the tiled passes over ONE segment,
// the whole lookup array [0, N), of global keys (row_base[t] + row; sentinel for invalid
// and outside-bag lookups, written with their positions by the keys kernel into (k_x,
// p_x)).  Passes ping-pong between (k_x, p_x) and (k_y, p_y); returns true when the sorted
// pairs end in (k_y, p_y).  Stable: equal keys stay in position order, as a stable
// device-wide radix sort leaves them.
template <typename IdxT, typename OffT, int DB>
bool launch_global_sort(const IdxT* idx, const OffT* off, const int64_t* row_base, int64_t N,
                        int bits, uint32_t* k_x, int32_t* p_x, uint32_t* k_y, int32_t* p_y,
                        uint32_t* hist, uint32_t sentinel, int32_t* err, const int32_t* bag_of,
                        hipStream_t st) {
  const int npass = (bits + DB - 1) / DB;
  TiledPass a{};
  a.row_base = row_base, a.T = 1, a.B = 1, a.hist = hist, a.sentinel = sentinel, a.err = err;
  a.bag_of = bag_of;
  a.J = (int)dlrm::ceil_div(N, (int64_t)kTile);
  a.global = 1;
  a.n_all = N;
  plan_scan_chunks(a);
  a.csum = hist + (size_t)a.J * (1 << DB);
  a.wide = a.J <= kWideScanMaxJ && (1 << DB) % 64 == 0 && dlrm::tuning(DLRM_TUNE_TBE_SORT) != 2;
  for (int ps = 0; ps < npass; ++ps) {
    const bool fwd = (ps & 1) == 0;  // x -> y on even passes
    a.shift = ps * DB;
    a.first = ps == 0;
    a.last = ps == npass - 1;
    a.kin = fwd ? k_x : k_y;
    a.pin = fwd ? p_x : p_y;
    a.kout = fwd ? k_y : k_x;
    a.pout = fwd ? p_y : p_x;
    hipLaunchKernelGGL((tbe_tiled_hist_kernel<IdxT, OffT, DB>), dim3(a.J), dim3(kTileThreads), 0,
                       st, idx, off, a);
    if (a.wide)
      hipLaunchKernelGGL((tbe_tiled_wide_scan_kernel<DB>), dim3((1 << DB) / 64),
                         dim3(kTileThreads), 0, st, a, static_cast<const void*>(off),
                         (int)sizeof(OffT) * 8);
    else if (a.C > 1)
      hipLaunchKernelGGL((tbe_tiled_csum_kernel<DB>), dim3(a.C), dim3(kTileThreads), 0, st, a,
                         static_cast<const void*>(off), (int)sizeof(OffT) * 8);
    if (!a.wide)
      hipLaunchKernelGGL((tbe_tiled_scan_kernel<DB>), dim3(a.C), dim3(kTileThreads), 0, st, a,
                         static_cast<const void*>(off), (int)sizeof(OffT) * 8);
    hipLaunchKernelGGL((tbe_tiled_scatter_kernel<IdxT, OffT, DB>), dim3(a.J), dim3(kScatThreads),
                       0, st, idx, off, a);
  }
  return (npass & 1) == 1;
}

template <typename KeyT>
struct BwdWs {
  KeyT* keys_in;
  KeyT* keys_out;
  int32_t* pos_in;
  int32_t* pos_out;
  int32_t* bag_of;
  float* partial;  // block partials; the sorts' digit histograms before the block kernel
  size_t partial_words;
  size_t total;
};

template <typename KeyT>
BwdWs<KeyT> carve_bwd_ws(void* base, int64_t N, int64_t D, int end_bit) {
  BwdWs<KeyT> w{};
  WsCarver c(base);
  w.keys_in = c.take<KeyT>(N);
  w.keys_out = c.take<KeyT>(N);
  w.pos_in = c.take<int32_t>(N);
  w.pos_out = c.take<int32_t>(N);
  w.bag_of = c.take<int32_t>(N);
  (void)end_bit;
  const size_t part = (size_t)2 * ((N + CH - 1) / CH) * D;
  // global sort, 10-bit digits: per-tile counts + the scan's chunk sums
  const size_t hist = (size_t)((N + kTile - 1) / kTile) * 1024 + (size_t)kMaxScanChunks * 1024;
  w.partial_words = part > hist ? part : hist;
  w.partial = c.take<float>(w.partial_words);
  w.total = c.used + 256;
  return w;
}

template <typename KeyT, typename IdxT, typename OffT>
int launch_bwd(int mode, float* W, float* mom, int64_t D, const int64_t* row_base, int T, int B,
               const void* idx, const void* off, int64_t N, int64_t total_rows, const float* psw,
               const float* gout, int64_t gbs, float lr, float eps, void* ws, size_t ws_bytes,
               int64_t max_seg, int32_t* err, int presorted, LaunchRole* defer, hipStream_t st,
               const char* name, bool sort_only = false) {
  if (defer) {  // until proven fusable: nothing deferred
    *defer = LaunchRole{};
    defer->magic = kRoleMagic;
  }
  if (N == 0) return DLRM_OK;
  const KeyT sentinel = (KeyT)total_rows;
  const int end_bit = bit_width_u64((uint64_t)total_rows);
  BwdWs<KeyT> w = carve_bwd_ws<KeyT>(ws, N, D, end_bit);
  DLRM_REQUIRE(ws_bytes >= w.total, DLRM_ERR_WORKSPACE, "%s: workspace %zu < required %zu",
               name, ws_bytes, w.total);
  const bool per_table = presort_applies(sizeof(KeyT), max_seg, N);
  // large tables (> kSegCap lookups): the tiled per-table sort, its digit histograms in the
  // block kernel's partial buffer (free until the sort is done)
  const int64_t tiles_j = dlrm::ceil_div(max_seg > 0 ? max_seg : 1, (int64_t)kTile);
  const int tdb = tiled_digit_bits(end_bit);  // the device-wide sort (global keys)
  // the tiled sort passes over each table's OWN key bits (pass_view): 10-bit digits never
  // need more passes than 8-bit ones there, and only the tables that need them run them
  const int64_t part_space = (int64_t)w.partial_words;
  // per-tile counts + the scan's chunk sums (at most kMaxScanChunks per table)
  const int64_t sort_words = (int64_t)T * (tiles_j + kMaxScanChunks);
  const int tdb_t = sort_words * (1 << 10) <= part_space ? 10 : tdb;
  const bool tiled = !per_table && sizeof(KeyT) == 4 && max_seg > kSegCap &&
                     N < (int64_t)0x7fffffff && (int64_t)T * tiles_j < (int64_t)INT32_MAX &&
                     sort_words * (1 << tdb_t) <= part_space &&
                     dlrm::tuning(DLRM_TUNE_TBE_SORT) != 1;
  // the tiled and global sorts carry each lookup's bag (not its position) when no
  // per-sample weights need the position: the block kernel then reads bags in sorted order
  const int32_t* bags = (!per_table && psw == nullptr) ? w.bag_of : nullptr;
  if (presorted == DLRM_PRESORTED_ANY || (per_table && presorted)) {
    // this batch's sort already ran: inside dlrm_tbe_forward_presort (per-table), or in
    // dlrm_tbe_backward_sort (any variant; the device-wide one ends in x or y by its parity)
    if (!per_table && !tiled && ((end_bit + tdb - 1) / tdb) % 2 == 0) {
      std::swap(w.keys_in, w.keys_out);
      std::swap(w.pos_in, w.pos_out);
    }
  } else if (per_table) {
    hipLaunchKernelGGL((tbe_bwd_segsort_kernel<IdxT, OffT>), dim3(T + 1), dim3(kSegThreads), 0,
                       st, static_cast<const IdxT*>(idx), static_cast<const OffT*>(off), row_base,
                       T, B, N, (uint32_t)sentinel, reinterpret_cast<uint32_t*>(w.keys_out),
                       w.pos_out, w.bag_of, err);
    DLRM_LAUNCH_CHECK(name);
  } else if (tiled) {
    const KeysArgs ka{row_base, T, B, N, (uint32_t)sentinel,
                      reinterpret_cast<uint32_t*>(w.keys_out), w.pos_out, w.bag_of, err,
                      keys_grid(T, B)};
    auto* ko = reinterpret_cast<uint32_t*>(w.keys_out);
    auto* ki = reinterpret_cast<uint32_t*>(w.keys_in);
    auto* hist = reinterpret_cast<uint32_t*>(w.partial);
    if (tdb_t == 10)
      launch_tiled_sort<IdxT, OffT, 10>(static_cast<const IdxT*>(idx),
                                        static_cast<const OffT*>(off), row_base, T, B,
                                        (int)tiles_j, end_bit, ki, w.pos_in, ko, w.pos_out, hist,
                                        (uint32_t)sentinel, err, (int)sizeof(OffT) * 8, bags, ka,
                                        st);
    else
      launch_tiled_sort<IdxT, OffT, 8>(static_cast<const IdxT*>(idx),
                                       static_cast<const OffT*>(off), row_base, T, B,
                                       (int)tiles_j, end_bit, ki, w.pos_in, ko, w.pos_out, hist,
                                       (uint32_t)sentinel, err, (int)sizeof(OffT) * 8, bags, ka,
                                       st);
    DLRM_LAUNCH_CHECK(name);
  } else {
    hipLaunchKernelGGL((tbe_bwd_keys_kernel<IdxT, OffT, KeyT, true>), dim3(keys_grid(T, B)),
                       dim3(256), 0, st, static_cast<const IdxT*>(idx),
                       static_cast<const OffT*>(off), row_base, T, B, N, sentinel, w.keys_in,
                       w.pos_in, w.bag_of, err);
    DLRM_LAUNCH_CHECK(name);
    auto* ki = reinterpret_cast<uint32_t*>(w.keys_in);
    auto* ko = reinterpret_cast<uint32_t*>(w.keys_out);
    auto* hist = reinterpret_cast<uint32_t*>(w.partial);
    const bool in_y =
        tdb == 10 ? launch_global_sort<IdxT, OffT, 10>(static_cast<const IdxT*>(idx),
                                                       static_cast<const OffT*>(off), row_base, N,
                                                       end_bit, ki, w.pos_in, ko, w.pos_out, hist,
                                                       (uint32_t)sentinel, err, bags, st)
                  : launch_global_sort<IdxT, OffT, 8>(static_cast<const IdxT*>(idx),
                                                      static_cast<const OffT*>(off), row_base, N,
                                                      end_bit, ki, w.pos_in, ko, w.pos_out, hist,
                                                      (uint32_t)sentinel, err, bags, st);
    DLRM_LAUNCH_CHECK(name);
    if (!in_y) {  // an even pass count left the sorted pairs in the input buffers
      std::swap(w.keys_in, w.keys_out);
      std::swap(w.pos_in, w.pos_out);
    }
  }

  if (sort_only) return DLRM_OK;

  const bool vec4 = (D % 4 == 0) &&
                    ((reinterpret_cast<uintptr_t>(W) & (mode == MODE_SGD_F16 ? 7 : 15)) == 0) &&
                    ((reinterpret_cast<uintptr_t>(gout) & 15) == 0) && (gbs % 4 == 0);
  const int64_t nchunks = vec4 ? D / 4 : D;
  int lpb = 1;
  while (lpb < nchunks && lpb < 64) lpb <<= 1;
  const int64_t maxv = dlrm::ceil_div(nchunks, lpb);
  DLRM_REQUIRE(maxv <= 8, DLRM_ERR_UNSUPPORTED, "%s: D=%lld too large", name, (long long)D);
  const int gpw = 64 / lpb;
  int ch = N >= kLongChN ? kLongCH : CH;
  const int64_t tch = dlrm::tuning(DLRM_TUNE_TBE_BLOCK);  // (sweeps / coverage tests)
  if (tch == CH || tch == kLongCH) ch = (int)tch;
  const int64_t nblocks = dlrm::ceil_div(N, (int64_t)ch);
  int64_t blocks = dlrm::ceil_div(dlrm::ceil_div(nblocks, gpw), 4);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  // the lean passes (4 gradient rows in flight per lane group at <= 128 VGPRs: twice the
  // resident waves of the 16-in-flight kernels, C1 block pass 100 -> ~65 us) wherever they
  // apply - deferred into later launches, or launched here
  if (sizeof(KeyT) == 4 && vec4 && maxv == 1 && (per_table || bags) &&
      tbe_role_fusable(mode, lpb, psw, (int64_t)B * gbs) &&
      (defer || dlrm::tuning(DLRM_TUNE_TBE_LEAN) != 1)) {
    LaunchRole local{};
    LaunchRole& r = defer ? *defer : local;
    r.W = W, r.mom = mom, r.psw = psw, r.gout = gout, r.partial = w.partial;
    r.keys = reinterpret_cast<const uint32_t*>(w.keys_out);
    r.pos = w.pos_out;
    r.bag_of = per_table ? w.bag_of : w.pos_out;
    r.D = D, r.gbs = gbs, r.N = N, r.lr = lr, r.eps = eps;
    r.sentinel = (uint32_t)sentinel;
    r.B = B, r.ch = ch, r.mode = mode, r.lpb = lpb;
    // a multiple of 8 workgroups keeps the co-launched GEMM tiles' XCD remap aligned
    r.blocks = (int32_t)(dlrm::ceil_div(blocks, (int64_t)8) * 8);
    r.kind = kRoleUpdate;
    r.magic = kRoleMagic;
    if (defer) return DLRM_OK;
    hipLaunchKernelGGL(tbe_update_pass_kernel<1>, dim3(r.blocks), dim3(256), 0, st, r);
    hipLaunchKernelGGL(tbe_update_pass_kernel<2>, dim3(r.blocks), dim3(256), 0, st, r);
    DLRM_LAUNCH_CHECK(name);
    return DLRM_OK;
  }
#define LAUNCH2(LPB, VW, MV, MODE)                                                             \
  do {                                                                                         \
    if (per_table || bags)                                                                     \
      hipLaunchKernelGGL((tbe_bwd_block_kernel<LPB, VW, MV, KeyT, MODE, true>), dim3(blocks),  \
                         dim3(256), 0, st, W, mom, D, B, w.keys_out, w.pos_out,                \
                         per_table ? w.bag_of : w.pos_out, psw, gout, gbs, N, lr, eps,         \
                         sentinel, w.partial, ch);                                             \
    else                                                                                       \
      hipLaunchKernelGGL((tbe_bwd_block_kernel<LPB, VW, MV, KeyT, MODE, false>), dim3(blocks), \
                         dim3(256), 0, st, W, mom, D, B, w.keys_out, w.pos_out, w.bag_of, psw, \
                         gout, gbs, N, lr, eps, sentinel, w.partial, ch);                      \
    hipLaunchKernelGGL((tbe_bwd_combine_kernel<LPB, VW, MV, KeyT, MODE>), dim3(blocks),        \
                       dim3(256), 0, st, W, mom, D, w.keys_out, N, lr, eps, sentinel,          \
                       w.partial, ch);                                                         \
  } while (0)
#define BY_LPB(VW, MODE)                             \
  switch (lpb) {                                     \
    case 1: LAUNCH2(1, VW, 1, MODE); break;          \
    case 2: LAUNCH2(2, VW, 1, MODE); break;          \
    case 4: LAUNCH2(4, VW, 1, MODE); break;          \
    case 8: LAUNCH2(8, VW, 1, MODE); break;          \
    case 16: LAUNCH2(16, VW, 1, MODE); break;        \
    case 32: LAUNCH2(32, VW, 1, MODE); break;        \
    default:                                         \
      if (maxv == 1) LAUNCH2(64, VW, 1, MODE);       \
      else if (maxv == 2) LAUNCH2(64, VW, 2, MODE);  \
      else if (maxv <= 4) LAUNCH2(64, VW, 4, MODE);  \
      else LAUNCH2(64, VW, 8, MODE);                 \
  }
#define BY_MODE(VW)                    \
  if (mode == MODE_SGD) {              \
    BY_LPB(VW, MODE_SGD)               \
  } else if (mode == MODE_ADAGRAD) {   \
    BY_LPB(VW, MODE_ADAGRAD)           \
  } else if (mode == MODE_SGD_F16) {   \
    BY_LPB(VW, MODE_SGD_F16)           \
  } else {                             \
    BY_LPB(VW, MODE_DENSE)             \
  }
  if (vec4) {
    BY_MODE(4)
  } else {
    BY_MODE(1)
  }
#undef BY_MODE
#undef BY_LPB
#undef LAUNCH2
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

int bwd_dispatch(int mode, float* W, float* mom, int64_t D, const int64_t* row_base, int T,
                 int B, const void* idx, int ib, const void* off, int ob, int64_t N,
                 int64_t total_rows, const float* psw, const float* gout, int64_t gbs, float lr,
                 float eps, void* ws, size_t ws_bytes, int64_t max_seg, int32_t* err,
                 int presorted, LaunchRole* defer, dlrm_stream_t stream, const char* name,
                 bool sort_only = false) {
  DLRM_ARG(((W && gout) || sort_only) && row_base && (N == 0 || (idx && off)),
           "%s: null pointer", name);
  DLRM_ARG(presorted >= 0 && presorted <= DLRM_PRESORTED_ANY, "%s: bad presorted %d", name,
           presorted);
  DLRM_ARG(T > 0 && B > 0 && D > 0 && N >= 0 && total_rows > 0, "%s: bad sizes", name);
  DLRM_ARG(ib == 32 || ib == 64, "%s: index_bits must be 32 or 64", name);
  DLRM_ARG(ob == 32 || ob == 64, "%s: offset_bits must be 32 or 64", name);
  DLRM_REQUIRE(N < (int64_t)INT32_MAX && (int64_t)T * B < (int64_t)INT32_MAX,
               DLRM_ERR_UNSUPPORTED, "%s: more than 2^31 lookups/bags per call", name);
  DLRM_ARG(gbs >= (int64_t)T * D, "%s: grad_batch_stride < T*D", name);
  DLRM_ARG(ws || N == 0, "%s: null workspace", name);
  hipStream_t st = dlrm::as_stream(stream);
  // 32-bit row keys: the sorts key on global rows (< 2^32 - 1 rows per call, e.g. 2^32
  // rows of D = 16 fp32 is 275 GB, beyond one GPU's table budget; shard across calls)
  DLRM_REQUIRE((uint64_t)total_rows < 0xFFFFFFFFull, DLRM_ERR_UNSUPPORTED,
               "%s: %lld rows in one call (at most 2^32 - 2)", name, (long long)total_rows);
#define BWD(K, I, O)                                                                     \
  return launch_bwd<K, I, O>(mode, W, mom, D, row_base, T, B, idx, off, N, total_rows, psw, \
                             gout, gbs, lr, eps, ws, ws_bytes, max_seg, err, presorted, defer, \
                             st, name, sort_only)
  if (ib == 32 && ob == 32) BWD(uint32_t, int32_t, int32_t);
  if (ib == 32 && ob == 64) BWD(uint32_t, int32_t, int64_t);
  if (ib == 64 && ob == 32) BWD(uint32_t, int64_t, int32_t);
  BWD(uint32_t, int64_t, int64_t);
#undef BWD
}

}  // namespace

extern "C" size_t dlrm_tbe_backward_workspace_size(int64_t num_lookups, int64_t total_rows,
                                                   int64_t D) {
  if (num_lookups <= 0) return 256;
  if (D < 1) D = 1;
  const int end_bit = bit_width_u64((uint64_t)(total_rows > 0 ? total_rows : 1));
  return carve_bwd_ws<uint32_t>(nullptr, num_lookups, D, end_bit).total;
}

extern "C" int dlrm_tbe_backward_sgd(float* weights, int64_t D, const int64_t* row_base,
                                     int32_t T, int32_t B, const void* indices,
                                     int32_t index_bits, const void* offsets,
                                     int32_t offset_bits, int64_t num_lookups,
                                     int64_t total_rows, const float* per_sample_weights,
                                     const float* grad_out, int64_t grad_batch_stride, float lr,
                                     int64_t max_lookups_per_table, void* workspace,
                                     size_t workspace_bytes, int32_t* error_flag,
                                     int32_t presorted, dlrm_stream_t stream) {
  return bwd_dispatch(MODE_SGD, weights, nullptr, D, row_base, T, B, indices, index_bits,
                      offsets, offset_bits, num_lookups, total_rows, per_sample_weights,
                      grad_out, grad_batch_stride, lr, 0.f, workspace, workspace_bytes,
                      max_lookups_per_table, error_flag, presorted, nullptr, stream,
                      "dlrm_tbe_backward_sgd");
}

extern "C" int dlrm_tbe_backward_sgd_f16(void* weights, int64_t D, const int64_t* row_base,
                                         int32_t T, int32_t B, const void* indices,
                                         int32_t index_bits, const void* offsets,
                                         int32_t offset_bits, int64_t num_lookups,
                                         int64_t total_rows, const float* per_sample_weights,
                                         const float* grad_out, int64_t grad_batch_stride,
                                         float lr, int64_t max_lookups_per_table,
                                         void* workspace, size_t workspace_bytes,
                                         int32_t* error_flag, int32_t presorted,
                                         dlrm_stream_t stream) {
  return bwd_dispatch(MODE_SGD_F16, static_cast<float*>(weights), nullptr, D, row_base, T, B,
                      indices, index_bits, offsets, offset_bits, num_lookups, total_rows,
                      per_sample_weights, grad_out, grad_batch_stride, lr, 0.f, workspace,
                      workspace_bytes, max_lookups_per_table, error_flag, presorted, nullptr, stream,
                      "dlrm_tbe_backward_sgd_f16");
}

extern "C" int dlrm_tbe_backward_rowwise_adagrad(
    float* weights, float* momentum, int64_t D, const int64_t* row_base, int32_t T, int32_t B,
    const void* indices, int32_t index_bits, const void* offsets, int32_t offset_bits,
    int64_t num_lookups, int64_t total_rows, const float* per_sample_weights,
    const float* grad_out, int64_t grad_batch_stride, float lr, float eps,
    int64_t max_lookups_per_table, void* workspace, size_t workspace_bytes, int32_t* error_flag,
    int32_t presorted, dlrm_stream_t stream) {
  DLRM_ARG(momentum, "dlrm_tbe_backward_rowwise_adagrad: null momentum");
  return bwd_dispatch(MODE_ADAGRAD, weights, momentum, D, row_base, T, B, indices, index_bits,
                      offsets, offset_bits, num_lookups, total_rows, per_sample_weights,
                      grad_out, grad_batch_stride, lr, eps, workspace, workspace_bytes,
                      max_lookups_per_table, error_flag, presorted, nullptr, stream,
                      "dlrm_tbe_backward_rowwise_adagrad");
}

extern "C" int dlrm_tbe_backward_dense(float* grad_weights, int64_t D, const int64_t* row_base,
                                       int32_t T, int32_t B, const void* indices,
                                       int32_t index_bits, const void* offsets,
                                       int32_t offset_bits, int64_t num_lookups,
                                       int64_t total_rows, const float* per_sample_weights,
                                       const float* grad_out, int64_t grad_batch_stride,
                                       int64_t max_lookups_per_table, void* workspace,
                                       size_t workspace_bytes, int32_t* error_flag,
                                       int32_t presorted, dlrm_stream_t stream) {
  return bwd_dispatch(MODE_DENSE, grad_weights, nullptr, D, row_base, T, B, indices, index_bits,
                      offsets, offset_bits, num_lookups, total_rows, per_sample_weights,
                      grad_out, grad_batch_stride, 0.f, 0.f, workspace, workspace_bytes,
                      max_lookups_per_table, error_flag, presorted, nullptr, stream,
                      "dlrm_tbe_backward_dense");
}

static_assert(sizeof(LaunchRole) <= sizeof(dlrm_launch_role), "dlrm_launch_role too small");

extern "C" int dlrm_tbe_backward_sort(int64_t D, const int64_t* row_base, int32_t T, int32_t B,
                                      const void* indices, int32_t index_bits,
                                      const void* offsets, int32_t offset_bits,
                                      int64_t num_lookups, int64_t total_rows,
                                      const float* per_sample_weights,
                                      int64_t max_lookups_per_table, void* workspace,
                                      size_t workspace_bytes, int32_t* error_flag,
                                      dlrm_stream_t stream) {
  return bwd_dispatch(MODE_SGD, nullptr, nullptr, D, row_base, T, B, indices, index_bits,
                      offsets, offset_bits, num_lookups, total_rows, per_sample_weights, nullptr,
                      (int64_t)T * D, 0.f, 0.f, workspace, workspace_bytes,
                      max_lookups_per_table, error_flag, 0, nullptr, stream,
                      "dlrm_tbe_backward_sort", true);
}

extern "C" int dlrm_tbe_backward_defer(
    int32_t mode, float* weights, float* momentum, int64_t D, const int64_t* row_base,
    int32_t T, int32_t B, const void* indices, int32_t index_bits, const void* offsets,
    int32_t offset_bits, int64_t num_lookups, int64_t total_rows,
    const float* per_sample_weights, const float* grad_out, int64_t grad_batch_stride, float lr,
    float eps, int64_t max_lookups_per_table, void* workspace, size_t workspace_bytes,
    int32_t* error_flag, int32_t presorted, dlrm_launch_role* role, dlrm_stream_t stream) {
  const char* name = "dlrm_tbe_backward_defer";
  DLRM_ARG(role, "%s: null role", name);
  DLRM_ARG(mode == 0 || mode == 1, "%s: mode must be 0 (sgd) or 1 (rowwise adagrad)", name);
  DLRM_ARG(mode == 0 || momentum, "%s: rowwise adagrad needs momentum", name);
  auto* r = reinterpret_cast<LaunchRole*>(role);
  *r = LaunchRole{};
  r->magic = kRoleMagic;
  return bwd_dispatch(mode == 0 ? MODE_SGD : MODE_ADAGRAD, weights, mode == 0 ? nullptr : momentum,
                      D, row_base, T, B, indices, index_bits, offsets, offset_bits, num_lookups,
                      total_rows, per_sample_weights, grad_out, grad_batch_stride, lr, eps,
                      workspace, workspace_bytes, max_lookups_per_table, error_flag, presorted, r,
                      stream, name);
}

extern "C" int32_t dlrm_role_blocks(const dlrm_launch_role* role) {
  const auto* r = reinterpret_cast<const LaunchRole*>(role);
  return r && r->magic == kRoleMagic ? r->blocks : 0;
}

namespace {

template <typename IdxT, typename OffT>
int launch_fwd_presort(const float* W, int64_t D, const int64_t* row_base, int T, int B,
                       const void* idx, const void* off, const float* psw, float* out,
                       int64_t out_bs, int64_t N, int64_t total_rows, void* ws, size_t ws_bytes,
                       int32_t* err, const MlpChain& mc, int mlp_blocks, bool sort,
                       hipStream_t st) {
  const char* name = "dlrm_tbe_forward_presort";
  BwdWs<uint32_t> w{};
  if (sort) {
    const int end_bit = bit_width_u64((uint64_t)total_rows);
    w = carve_bwd_ws<uint32_t>(ws, N, D, end_bit);
    DLRM_REQUIRE(ws_bytes >= w.total, DLRM_ERR_WORKSPACE, "%s: workspace %zu < required %zu",
                 name, ws_bytes, w.total);
  }
  const int nsort = sort ? T + 1 : 0;
  const bool vec4 = (D % 4 == 0) && ((reinterpret_cast<uintptr_t>(W) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(out) & 15) == 0) && (out_bs % 4 == 0);
  const int64_t nchunks = vec4 ? D / 4 : D;
  int lpb = 1;
  while (lpb < nchunks && lpb < 64) lpb <<= 1;
  const int64_t maxv = dlrm::ceil_div(nchunks, lpb);
  DLRM_REQUIRE(maxv <= 8, DLRM_ERR_UNSUPPORTED, "%s: D=%lld too large", name, (long long)D);
  const int64_t nbags = (int64_t)T * B;
  const int gpw = 64 / lpb;
  int64_t gblocks = dlrm::ceil_div(dlrm::ceil_div(nbags, gpw), kPreThreads / 64);
  if (gblocks > 8192) gblocks = 8192;
  if (gblocks < 1) gblocks = 1;
  if (!out) gblocks = 0;  // the lookup is fused into its consumer (interaction gather)
  const dim3 grid((unsigned)(nsort + mlp_blocks + gblocks)), block(kPreThreads);
  const IdxT* ip = static_cast<const IdxT*>(idx);
  const OffT* op = static_cast<const OffT*>(off);
  const uint32_t sentinel = (uint32_t)total_rows;
#define PRE(LPB, VW, MV)                                                                         \
  hipLaunchKernelGGL((tbe_fwd_presort_kernel<LPB, VW, MV, IdxT, OffT>), grid, block, 0, st, W, D, \
                     row_base, T, B, ip, op, psw, out, out_bs, err, N, sentinel,                  \
                     reinterpret_cast<uint32_t*>(w.keys_out), w.pos_out, w.bag_of, mc,       \
                     mlp_blocks, nsort)
#define PRE_LPB(VW)                        \
  switch (lpb) {                           \
    case 1: PRE(1, VW, 1); break;          \
    case 2: PRE(2, VW, 1); break;          \
    case 4: PRE(4, VW, 1); break;          \
    case 8: PRE(8, VW, 1); break;          \
    case 16: PRE(16, VW, 1); break;        \
    case 32: PRE(32, VW, 1); break;        \
    default:                               \
      if (maxv == 1) PRE(64, VW, 1);       \
      else if (maxv == 2) PRE(64, VW, 2);  \
      else if (maxv <= 4) PRE(64, VW, 4);  \
      else PRE(64, VW, 8);                 \
  }
  if (vec4) {
    PRE_LPB(4)
  } else {
    PRE_LPB(1)
  }
#undef PRE_LPB
#undef PRE
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

}  // namespace

extern "C" int dlrm_tbe_forward_presort(const float* weights, int64_t D, const int64_t* row_base,
                                        int32_t T, int32_t B, const void* indices,
                                        int32_t index_bits, const void* offsets,
                                        int32_t offset_bits, const float* per_sample_weights,
                                        float* out, int64_t out_batch_stride,
                                        int64_t num_lookups, int64_t total_rows,
                                        int64_t max_lookups_per_table, void* workspace,
                                        size_t workspace_bytes, int32_t* error_flag,
                                        const dlrm_mlp_chain* bottom, dlrm_stream_t stream) {
  const char* name = "dlrm_tbe_forward_presort";
  MlpChain mc{};
  int mlp_blocks = 0;
  if (bottom) {
    DLRM_ARG(mlp_chain_prepare(bottom, mc), "%s: unsupported bottom MLP chain", name);
    mlp_blocks = (int)mlp_chain_blocks(mc);
  }
  const bool sort = presort_applies((uint64_t)total_rows < 0xFFFFFFFFull ? 4 : 8,
                                    max_lookups_per_table, num_lookups) &&
                    num_lookups > 0 && T * (int64_t)B < INT32_MAX;
  // no per-table sort (the backward sorts itself) but a bottom MLP to run: one launch of
  // the lookup and the MLP roles (D <= 512 keeps the gather within its 8 chunks per lane)
  const bool pair = !sort && bottom && out && num_lookups > 0 && T * (int64_t)B < INT32_MAX &&
                    D <= 512;
  if (!sort && !pair) {
    DLRM_REQUIRE(out, DLRM_ERR_UNSUPPORTED,
                 "%s: out = NULL needs the per-table sort (32-bit keys, bounded tables)", name);
    const int rc = dlrm_tbe_forward(weights, D, row_base, T, B, indices, index_bits, offsets,
                                    offset_bits, per_sample_weights, out, out_batch_stride,
                                    error_flag, stream);
    if (rc != DLRM_OK || !bottom) return rc;
    return dlrm_mlp_chain_forward(bottom, stream);
  }
  DLRM_ARG(weights && row_base && offsets && indices, "%s: null pointer", name);
  DLRM_ARG(T > 0 && B > 0 && D > 0 && total_rows > 0, "%s: bad sizes", name);
  DLRM_ARG(index_bits == 32 || index_bits == 64, "%s: index_bits must be 32|64", name);
  DLRM_ARG(offset_bits == 32 || offset_bits == 64, "%s: offset_bits must be 32|64", name);
  DLRM_ARG(out_batch_stride >= (int64_t)T * D, "%s: out_batch_stride < T*D", name);
  DLRM_ARG(workspace || !sort, "%s: null workspace", name);
  hipStream_t st = dlrm::as_stream(stream);
#define PS(I, O)                                                                           \
  return launch_fwd_presort<I, O>(weights, D, row_base, T, B, indices, offsets,            \
                                  per_sample_weights, out, out_batch_stride, num_lookups,  \
                                  total_rows, workspace, workspace_bytes, error_flag, mc,  \
                                  mlp_blocks, sort, st)
  if (index_bits == 32 && offset_bits == 32) PS(int32_t, int32_t);
  if (index_bits == 32) PS(int32_t, int64_t);
  if (offset_bits == 32) PS(int64_t, int32_t);
  PS(int64_t, int64_t);
#undef PS
}

extern "C" int dlrm_mlp_chain_supported(const dlrm_mlp_chain* chain) {
  MlpChain mc{};
  return mlp_chain_prepare(chain, mc);
}

extern "C" int dlrm_mlp_chain_forward(const dlrm_mlp_chain* chain, dlrm_stream_t stream) {
  const char* name = "dlrm_mlp_chain_forward";
  MlpChain mc{};
  DLRM_ARG(mlp_chain_prepare(chain, mc), "%s: unsupported chain", name);
  if (chain->rows == 0) return DLRM_OK;
  hipLaunchKernelGGL(mlp_chain_kernel, dim3((unsigned)mlp_chain_blocks(mc)),
                     dim3(kMlpWaves * 64), 0, dlrm::as_stream(stream), mc);
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}
