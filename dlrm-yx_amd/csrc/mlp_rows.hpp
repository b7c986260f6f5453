// Row-block MLP forward: the bottom MLP of the DLRM step (DLRM_Net.apply_mlp over
// create_mlp's Linear+ReLU stack, dlrm_s_pytorch.py:227-265, 518-524) for 16 samples per
// workgroup, every layer in one pass with the activations kept in LDS.
//
// The bottom MLP is short and narrow (C3: 13 -> 512 -> 256 -> 128 on 2048 samples), so as
// three GEMM launches it is latency-bound (~25 us for 0.7 GFLOP).  Here a workgroup owns 16
// rows: it stages their inputs in LDS, and each of its 8 waves computes 16-column tiles of
// the next activation on v_mfma_f32_16x16x4_f32 (A = the LDS rows, B = weight rows read
// straight from global/L2 as float4, three 16-k chunks ahead), applies ReLU, writes the tile
// to the layer's activation buffer (needed by the backward) and into the other LDS
// buffer as the next layer's input (bias column = 1, zero padding).  No inter-workgroup
// traffic: the role runs beside the TBE lookup and the backward's index sort inside one
// launch (tbe_bwd.hip), or alone (dlrm_mlp_chain_forward).
//
// Bias folding as in the trainer: layer l's input has in_width[l] columns; for l > 0,
// column out_width[l-1] is the constant 1 and the rest of the padding is 0; W_l is
// [out_width[l], >= in_width[l]] with the bias in the bias column.
#pragma once
#include "common.hpp"
#include "dlrm_hip.h"

namespace {

constexpr int kMlpRows = 16;      // samples per workgroup
constexpr int kMlpWaves = 16;     // waves per workgroup (1024 threads)
constexpr int kMlpTiles = 2;      // 16-column tiles per wave: out_width <= 16 * 2 * 16 = 512
static_assert(kMlpTiles == 2, "mlp_rows_body dispatches mlp_kloop<1..2>");
constexpr int kMlpMaxK = 528;     // input width rounded to 16, LDS capacity
constexpr int kMlpPitch = kMlpMaxK + 4;
constexpr int kMlpLdsFloats = 2 * kMlpRows * kMlpPitch + 4;  // + the split chain's flag

using mlp_f32x4 = __attribute__((ext_vector_type(4))) float;

struct MlpChain {
  int layers;
  int64_t rows;
  const float* X;
  int64_t ldx;
  int kin[DLRM_MLP_MAX_LAYERS];
  int nout[DLRM_MLP_MAX_LAYERS];
  const float* W[DLRM_MLP_MAX_LAYERS];
  int64_t ldw[DLRM_MLP_MAX_LAYERS];
  float* Y[DLRM_MLP_MAX_LAYERS];
  int64_t ldy[DLRM_MLP_MAX_LAYERS];
  int parts;     // workgroups per 16-row block (1, 2, 4)
  int split;     // the layer whose column tiles the parts share
  int* tickets;  // per row block (parts > 1, split < layers - 1)
};

// K loop of one layer for this wave's NTW column tiles: acc[j] += A(16 x kp) . W_tile^T.
// A fragments come from LDS (row l16, k = 16c + 4kq .. +3, read one chunk ahead); B
// fragments are raw buffer loads of W[col][16c + 4kq .. +3] kept in a ring of kMlpRing
// register sets (chunks c+1 .. c+kMlpRing-1 in flight under chunk c's MFMAs: one chunk is
// only 4 * NTW MFMAs, ~130-260 cycles, while a weight fetch from a loaded L2 / the MALL
// takes 500-2000 cycles - a 4-deep ring left the role latency-bound).  An out-of-range
// float4 (column >= n or k >= in_width) gets an offset past the descriptor's extent and
// reads as zeros, so a fetched register is never touched before its MFMA.
constexpr int kMlpRing = 8;

// Tiles tb + wave + j * kMlpWaves (j < NTW).
template <int NTW>
__device__ __forceinline__ void mlp_kloop(mlp_f32x4 (&acc)[kMlpTiles], const float* in,
                                          __amdgpu_buffer_rsrc_t rw, int tb, int wave, int n,
                                          int kp, int64_t ldw, int nch, int l16, int kq) {
  constexpr int P = kMlpPitch, NW = kMlpWaves, R = kMlpRing;
  auto fetch = [&](int c, float4 (&bv)[NTW]) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int col = (tb + wave + j * NW) * 16 + l16, k = c * 16 + 4 * kq;
      const int off = (col < n && k < kp) ? (int)((col * ldw + k) * 4) : 0x7ffffff0;
      bv[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 0));
    }
  };
  // a chunk wholly inside the row (16 c + 16 <= kp, uniform): the lane's chunk-0 offset (or a
  // past-the-end one for a column >= n) in the VGPR, the chunk's advance in the scalar
  // offset - no per-load VALU (the masked form above costs ~6 per load)
  int voff[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int col = (tb + wave + j * NW) * 16 + l16;
    voff[j] = col < n ? (int)((col * ldw + 4 * kq) * 4) : 0x7ffffff0;
  }
  auto fetch_fast = [&](int c, float4 (&bv)[NTW]) {
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      bv[j] = __builtin_bit_cast(float4,
                                 __builtin_amdgcn_raw_buffer_load_b128(rw, voff[j], c * 64, 0));
  };
  auto lda = [&](int c) {
    return *reinterpret_cast<const float4*>(in + l16 * P + c * 16 + 4 * kq);
  };
  float4 a = lda(0);
  auto step = [&](int c, const float4 (&bv)[NTW]) {
    const float4 an = lda(c + 1 < nch ? c + 1 : c);
    // k-step outer, tile inner: consecutive MFMAs use different accumulators
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bv[j].x, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bv[j].y, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bv[j].z, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bv[j].w, acc[j], 0, 0, 0);
    a = an;
  };
  float4 ring[R][NTW];
#pragma unroll
  for (int u = 0; u < R - 1; ++u)
    if (u < nch) fetch(u, ring[u]);
  for (int c0 = 0; c0 < nch; c0 += R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int c = c0 + u;
      if (c >= nch) break;
      if (c + R - 1 < nch) {
        if ((c + R) * 16 <= kp)
          fetch_fast(c + R - 1, ring[(u + R - 1) % R]);
        else
          fetch(c + R - 1, ring[(u + R - 1) % R]);
      }
      step(c, ring[u]);
    }
  }
}

// Split chains (mc.parts > 1): workgroup blk is part q = blk % parts of row block
// blk / parts.  Layers before mc.split run whole in every part (part 0 writes their Y);
// layer mc.split covers this part's tiles [tb, te) only; if more layers follow, the
// outputs are published write-through (sc1 stores, drained, then an agent-scope ticket -
// the MI355X guide's cross-XCD form, as in gemm.hip's split-K) and the last part to
// arrive reads the others' columns back (sc1 loads) and runs the remaining layers.
__device__ __forceinline__ void mlp_rows_body(const MlpChain& mc, int64_t blk, float* lds) {
  constexpr int RB = kMlpRows, P = kMlpPitch, NW = kMlpWaves, MT = kMlpTiles;
  constexpr int NT = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar tile tests
  const int kq = lane >> 4, l16 = lane & 15;
  const int parts = mc.parts > 1 ? mc.parts : 1;
  const int64_t rblk = blk / parts;
  const int q = (int)(blk - rblk * parts);
  const int64_t r0 = rblk * RB;
  float* in = lds;
  float* nx = lds + RB * P;
  {  // layer 0 input: X rows, zero-padded to a multiple of 16 columns
    const int kp = mc.kin[0], kr4 = ((kp + 15) & ~15) / 4;
    for (int e = tid; e < RB * kr4; e += NT) {
      const int r = e / kr4, c4 = e - r * kr4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r0 + r < mc.rows && 4 * c4 < kp)
        v = *reinterpret_cast<const float4*>(mc.X + (r0 + r) * mc.ldx + 4 * c4);
      *reinterpret_cast<float4*>(in + r * P + 4 * c4) = v;
    }
  }
  __syncthreads();
  for (int l = 0; l < mc.layers; ++l) {
    const int kp = mc.kin[l], n = mc.nout[l];
    const int nch = (kp + 15) / 16, ntile = (n + 15) / 16;
    const float* W = mc.W[l];
    const int64_t ldw = mc.ldw[l];
    // raw buffer loads over exactly W's rows (mlp_kloop)
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)W, (short)0, (int)(((int64_t)(n - 1) * ldw + kp) * 4), 0x00020000);
    const bool split = parts > 1 && l == mc.split;
    const bool publish = split && l + 1 < mc.layers;  // the last part continues
    const int tb = split ? q * ntile / parts : 0, te = split ? (q + 1) * ntile / parts : ntile;
    const int mt = te - tb;  // this part's tiles
    mlp_f32x4 acc[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[j] = mlp_f32x4{0.f, 0.f, 0.f, 0.f};
    const int nt_w = mt > wave ? (mt - wave + NW - 1) / NW : 0;  // this wave's tiles
    // the tile count is a template argument of the K loop: no branch inside it, so the
    // compiler's vmcnt accounting keeps the prefetched chunks in flight
    switch (nt_w) {
      case 1: mlp_kloop<1>(acc, in, rw, tb, wave, n, kp, ldw, nch, l16, kq); break;
      case 2: mlp_kloop<2>(acc, in, rw, tb, wave, n, kp, ldw, nch, l16, kq); break;
      default: break;
    }
    // epilogue: ReLU; register r of a 16x16 accumulator = row 4*kq + r, column l16
    float* Y = mc.Y[l];
    const int64_t ldy = mc.ldy[l];
    const bool write_y = q == 0 || l >= mc.split;  // replicated layers: part 0 writes
    const int64_t nrow = mc.rows - r0 < RB ? mc.rows - r0 : RB;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Y + r0 * ldy), (short)0, (int)(publish ? nrow * ldy * 4 : 0), 0x00020000);
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int col = (tb + wave + j * NW) * 16 + l16;
      if (wave + j * NW < mt && col < n) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * kq + r;
          const float v = fmaxf(acc[j][r], 0.f);
          nx[row * P + col] = v;
          if (publish) {  // write-through (sc1): read back by the last part to arrive
            if (row < nrow)
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), ry,
                                                    (int)((row * ldy + col) * 4), 0, 16);
          } else if (write_y && r0 + row < mc.rows) {
            Y[(r0 + row) * ldy + col] = v;
          }
        }
      }
    }
    if (publish) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = reinterpret_cast<int*>(lds + 2 * RB * P);  // past both activation buffers
      // The hand-off is the MI355X guide's write-through form (cdna_hip_programming.md §6,
      // Guideline 16): every store of the handed-off columns is sc1 and drained (vmcnt(0),
      // barrier) before the relaxed agent-scope ticket, and every load of them below is an
      // sc1 buffer load, issued after the barrier that broadcasts "last" - valid in place of a
      // release/acquire pair for any placement of the parts on XCDs, and cheaper (no L2
      // writeback / invalidate).  gemm.hip's split-K completion is the same protocol.
      if (tid == 0) {
        const int t = __hip_atomic_fetch_add(mc.tickets + rblk, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        const int last = t == parts - 1;
        if (last) __hip_atomic_store(mc.tickets + rblk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *reinterpret_cast<volatile int*>(flag) = last;
      }
      __syncthreads();
      if (!*reinterpret_cast<volatile int*>(flag)) return;
      // the other parts' columns of this block's rows (sc1 loads; rows past the batch: 0)
      const int c0 = tb * 16, c1 = te * 16 < n ? te * 16 : n, other = n - (c1 - c0);
      for (int e = tid; e < RB * other; e += NT) {
        const int row = e / other, k = e - row * other;
        const int col = k < c0 ? k : k + (c1 - c0);
        float v = 0.f;
        if (row < nrow)
          v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            ry, (int)((row * ldy + col) * 4), 0, 16));
        nx[row * P + col] = v;
      }
    }
    if (l + 1 < mc.layers) {  // next input: bias column 1, zeros to the 16-column boundary
      const int kr = (mc.kin[l + 1] + 15) & ~15, extra = kr - n;
      for (int e = tid; e < RB * extra; e += NT) {
        const int r = e / extra, c = n + (e - r * extra);
        nx[r * P + c] = c == n ? 1.f : 0.f;
      }
    }
    __syncthreads();
    float* t = in;
    in = nx;
    nx = t;
  }
}

// Host-side check + conversion (the ABI struct -> kernel argument).
inline int mlp_chain_prepare(const dlrm_mlp_chain* c, MlpChain& mc) {
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!c || c->layers < 1 || c->layers > DLRM_MLP_MAX_LAYERS || c->rows < 0) return 0;
  if (!c->X || !a16(c->X) || c->ldx % 4 != 0) return 0;
  mc.layers = c->layers;
  mc.rows = c->rows;
  mc.X = c->X;
  mc.ldx = c->ldx;
  for (int l = 0; l < c->layers; ++l) {
    const int64_t kin = c->in_width[l], n = c->out_width[l];
    if (kin < 1 || kin % 4 != 0 || ((kin + 15) & ~15) > kMlpMaxK) return 0;
    if (n < 1 || n > kMlpWaves * kMlpTiles * 16) return 0;
    if (l == 0 ? c->ldx < kin : kin != ((c->out_width[l - 1] + 1 + 3) / 4) * 4) return 0;
    if (!c->W[l] || !a16(c->W[l]) || c->ldw[l] % 4 != 0 || c->ldw[l] < kin) return 0;
    if (((n - 1) * c->ldw[l] + kin) * 4 >= 0x7ff00000LL) return 0;  // 32-bit buffer offsets
    if (!c->Y[l] || c->ldy[l] < n) return 0;
    mc.kin[l] = (int)kin;
    mc.nout[l] = (int)n;
    mc.W[l] = c->W[l];
    mc.ldw[l] = c->ldw[l];
    mc.Y[l] = c->Y[l];
    mc.ldy[l] = c->ldy[l];
  }
  mc.parts = c->parts > 1 ? c->parts : 1;
  mc.split = c->split_layer;
  mc.tickets = c->tickets;
  if (mc.parts > 1) {
    if (mc.parts != 2 && mc.parts != 4) return 0;
    if (mc.split < 0 || mc.split >= c->layers) return 0;
    if ((c->out_width[mc.split] + 15) / 16 < mc.parts) return 0;  // a tile per part
    if (mc.split + 1 < c->layers) {
      if (!c->tickets) return 0;
      if ((int64_t)kMlpRows * c->ldy[mc.split] * 4 >= 0x7ff00000LL) return 0;  // 32-bit offsets
    }
  }
  return 1;
}

// Workgroups of the forward chain: parts per 16-row block.
inline int64_t mlp_chain_blocks(const MlpChain& mc) {
  return ((mc.rows + kMlpRows - 1) / kMlpRows) * mc.parts;
}

}  // namespace
