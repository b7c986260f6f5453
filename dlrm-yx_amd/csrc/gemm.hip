// Exact-fp32 GEMM with fused epilogues on the gfx950 fp32 matrix core
// (v_mfma_f32_16x16x4_f32 / 32x32x2_f32: 64 FLOP/clk/SIMD, k-ordered fmaf chain, no xf32).
//
// Serves the DLRM MLPs (DLRM_Net.create_mlp / apply_mlp, dlrm_s_pytorch.py:227-265,
// 518-524): Linear forward with bias(+ReLU) fused, dgrad with the ReLU mask of the
// previous activation fused, wgrad with the SGD update fused (single GPU) or stored
// into the flat gradient bucket (multi GPU, all-reduced before the update).
//
// Main kernel (gemm_group_kernel): up to four INDEPENDENT GEMMs in one launch (a grouped
// GEMM: e.g. the dgrad of layer l beside the wgrad of layer l+1, which read the same
// gradient and write different buffers), each with its own operand layout, epilogue and
// K split.  Workgroups are 256 threads = 4 waves in a 2x2 arrangement, each wave owning
// a (BM/2)x(BN/2) sub-tile of 16x16 accumulators, software-pipelined over BK = 32:
//   * the fragments of K-tile t are in registers before its MFMAs start;
//   * while tile t multiplies, tile t+1 (fetched one iteration earlier) is written to the
//     other LDS buffer one float4 per k-step and each freed register is refilled with
//     tile t+2 (raw buffer loads: out-of-range float4s read as zeros, no branches);
//   * one barrier per K-tile, then tile t+1's fragments are read under the last k-step.
// The k-order inside a K-tile is permuted so a lane's operands are CONTIGUOUS: an
// operand that is k-contiguous in HBM (X rows, nn.Linear W rows) is staged [mn][k] and
// read with ds_read_b128; an mn-contiguous one is staged [k][mn] and read with
// conflict-free ds_read_b32.  The grid is remapped bijectively so each XCD (private
// 4 MiB L2) receives a contiguous run of blocks: neighbouring tiles of one problem, and
// all the K splits of one tile.
//
// Bias as a row sum: the wgrad of a Linear layer with its bias stored as an extra weight
// column (bias folding, trainer layout) needs db[m] = sum_k dY(k, m) = (op(A) . 1)[m].
// With ones_col >= 0 the kernel accumulates the A fragments it already holds (one VALU
// add per fragment, beside the MFMAs) and writes C[m][ones_col] = epi(alpha * db[m]), so
// N stays the weight width (1024, not 1028: no mostly-empty 17th column of tiles).
//
// Split-K inside the launch: split workgroups store their fp32 partial tile (and row
// sums) into a per-(tile, split) record in fragment order (every lane writes and reads
// 64 contiguous bytes); the LAST workgroup of a tile to finish (agent-scope ticket) sums
// the records IN SPLIT ORDER - deterministic, and bitwise the sum a separate reduce over
// s = 0..S-1 would give - and applies the epilogue.  No reduce launch.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.hpp"
#include "tbe_bwd_roles.hpp"

// Timeline hook of the pipelined body (tools/gemm_lab.hip defines it to stamp the clock at
// the prologue, every K-tile and the epilogue; empty in the library).
#ifndef DLRM_GEMM_STAMP
#define DLRM_GEMM_STAMP(slot)
#endif

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kThreads = 256;
constexpr int kMaxSplit = 32;
constexpr int kMaxGroup = 6;
constexpr int64_t kTicketCap = 16384;  // int32 tickets in the fixed 64 KiB workspace head
constexpr int kBK = 32;
constexpr int kRasterRows = 4;  // tile rows per raster group (pipe_body; 8 and 16 slower at C3,
                                 // profiles/r06_raster_rows_ab.txt)

struct GemmParams {
  int64_t M, N, K;
  float alpha;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int epi;
  const float* bias;
  const float* aux;
  int64_t ldaux;
  int64_t ones_col;  // >= 0: C[m][ones_col] = epi(alpha * sum_k op(A)(m, k))
  int layout;        // 0: A,B k-contiguous  1: A k-contig, B mn  2: A,B mn  3: A mn, B k-contig
  int tiles_m, tiles_n;
  int splits;        // K splits per output tile (1 = no split)
  int block0;        // first (virtual) block of this problem in its launch
  int64_t kchunk;    // K range per split (multiple of kBK)
  float* ws;         // split records [tile][split][BM*BN + BM] (splits > 1)
  int* counters;     // per-tile arrival tickets (splits > 1; zero between launches)
  int mode;          // DLRM_GEMM_FULL / _PARTIAL (split partials -> part) / _REDUCE
  float* part;       // PARTIAL/REDUCE: [splits][M][N] fp32, then [splits][M] row sums
};

struct GemmGroup {
  GemmParams p[kMaxGroup];
  int n;
  int total;  // blocks in the launch
};

// Row swizzle of a k-contiguous [mn][32] LDS image (16-B chunk c of row r stored at chunk
// c ^ swz_kc(r)): the 16-lane groups of a fragment's ds_read_b128 (lanes l16 x k-quarter kq,
// chunks 2kq + h) then cover all 64 banks.  An mn-contiguous [32][MN] image flips bit 4 of
// mn on k-rows 8..15 and 24..31 instead (the two k-quarters of a ds_read_b32 half-wave land
// on opposite 16-bank halves).
__device__ __forceinline__ int swz_kc(int r) {
  return ((r >> 1) & 7) ^ (((unsigned)((r & 15) - 4) < 8u) ? 2 : 0);
}

// One operand's (MN x BKT) panel, staged global -> registers -> LDS.
//   KC  : X(mn, k) = X[mn*ld + k]  -> LDS [mn][BKT + 4]   (fragments: ds_read_b128)
//   !KC : X(mn, k) = X[k*ld + mn]  -> LDS [BKT][MN + 4]   (fragments: ds_read_b32)
// SWZ (BKT = 32, MN >= 32): unpadded and swizzled as above - no bank conflicts in the
// fragment reads of the pipelined body (the padded images read 2-way conflicted: +4 % on
// the C3 step, profiles/r05_gemm_swizzle_ab.txt).
template <int MN, int BKT, bool KC, bool VEC, int NT, bool SWZ = false>
struct Stage {
  static_assert(!SWZ || (BKT % 32 == 0 && MN >= 32), "swizzled images: BKT 32 U, MN >= 32");
  static constexpr int PITCH = SWZ ? (KC ? 32 : MN) : (KC ? BKT + 4 : MN + 4);
  // floats per LDS buffer (swizzled KC: BKT / 32 sub-images [MN][32], one per 32-deep
  // sub-tile, each laid out exactly as the BKT = 32 image)
  static constexpr int SIZE = SWZ ? MN * BKT : (KC ? MN * PITCH : BKT * PITCH);
  // float offset of element (mn, k) in the image (KC: k % 4 == 0 addresses a whole chunk)
  __device__ __forceinline__ static int at(int mn, int k) {
    if constexpr (!SWZ) return KC ? mn * PITCH + k : k * PITCH + mn;
    else if constexpr (KC)
      return ((k >> 5) * MN + mn) * 32 + 4 * (((k & 31) >> 2) ^ swz_kc(mn)) + (k & 3);
    else return k * PITCH + (mn ^ (((k >> 3) & 1) << 4));
  }
  static constexpr int NV = MN * BKT / 4 / NT;               // float4 per thread
  static_assert(NV >= 1 && MN * BKT % (4 * NT) == 0, "panel / thread mismatch");
  float4 regs[NV];

  __device__ __forceinline__ void coords(int q, int& mn, int& k) const {
    if constexpr (KC && SWZ) {  // sub-image, then row, then 8 chunks of a 32-deep row
      const int u = q / (MN * 8), r = q - u * (MN * 8);
      mn = r >> 3;
      k = 32 * u + 4 * (r & 7);
    } else if constexpr (KC) {
      mn = q / (BKT / 4);
      k = 4 * (q % (BKT / 4));
    } else {
      k = q / (MN / 4);
      mn = 4 * (q % (MN / 4));
    }
  }

  __device__ __forceinline__ void load(const float* __restrict__ X, int64_t ld, int64_t mn0,
                                       int64_t mnlim, int64_t k0, int64_t klim, int tid) {
    if (VEC && mn0 + MN <= mnlim && k0 + BKT <= klim) {  // workgroup-uniform fast path
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        int mn, k;
        coords(tid + v * NT, mn, k);
        const float* ptr = KC ? X + (mn0 + mn) * ld + k0 + k : X + (k0 + k) * ld + mn0 + mn;
        regs[v] = *reinterpret_cast<const float4*>(ptr);
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int mn, k;
      coords(tid + v * NT, mn, k);
      const int64_t gmn = mn0 + mn, gk = k0 + k;
      const float* ptr = KC ? X + gmn * ld + gk : X + gk * ld + gmn;
      const bool full = KC ? (gmn < mnlim && gk + 3 < klim) : (gk < klim && gmn + 3 < mnlim);
      if (VEC && full) {
        regs[v] = *reinterpret_cast<const float4*>(ptr);
      } else {
        float e[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const bool ok = KC ? (gmn < mnlim && gk + c < klim) : (gk < klim && gmn + c < mnlim);
          e[c] = ok ? ptr[c] : 0.f;
        }
        regs[v] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  }

  // Single float4 v of the panel (pipelined kernel): `fast` = whole panel in range.
  __device__ __forceinline__ void load_one(int v, const float* __restrict__ X, int64_t ld,
                                           int64_t mn0, int64_t mnlim, int64_t k0, int64_t klim,
                                           int tid, bool fast) {
    int mn, k;
    coords(tid + v * NT, mn, k);
    const int64_t gmn = mn0 + mn, gk = k0 + k;
    const float* ptr = KC ? X + gmn * ld + gk : X + gk * ld + gmn;
    if (VEC && fast) {
      regs[v] = *reinterpret_cast<const float4*>(ptr);
      return;
    }
    float e[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool ok = KC ? (gmn < mnlim && gk + c < klim) : (gk < klim && gmn + c < mnlim);
      e[c] = ok ? ptr[c] : 0.f;
    }
    regs[v] = make_float4(e[0], e[1], e[2], e[3]);
  }

  // Branch-free variant for the pipelined kernel: a raw buffer load (32-bit offsets from
  // a wave-uniform descriptor) whose out-of-range lanes get an offset past the descriptor's
  // extent, so the hardware returns zeros.  Requires 4-element granularity (K % 4 == 0 for
  // k-contiguous operands, the mn extent % 4 == 0 otherwise, 16-B aligned rows) so a
  // float4 is entirely in or out of range.  Every call issues exactly one
  // buffer_load_dwordx4 (static vmcnt accounting, no exec-masked branches).
  __device__ __forceinline__ void load_one4(int v, __amdgpu_buffer_rsrc_t rsrc, int64_t ld,
                                            int64_t mn0, int64_t mnlim, int64_t k0, int64_t klim,
                                            int tid) {
    int mn, k;
    coords(tid + v * NT, mn, k);
    const int64_t gmn = mn0 + mn, gk = k0 + k;
    const bool ok = gmn < mnlim && gk < klim;
    const int64_t e = KC ? gmn * ld + gk : gk * ld + gmn;
    const int off = ok ? (int)(e * 4) : 0x7ffffff0;
    const auto t = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
    regs[v] = __builtin_bit_cast(float4, t);
  }

  // Pipelined fetch with per-thread offsets precomputed once (32-bit, bytes, at K-tile 0 of
  // the split) so a K-tile costs one add + one compare per float4.  Out-of-range float4s
  // read as zeros: rows/columns past the operand are outside the buffer descriptor except
  // (KC) the columns k >= K of a row and (!KC) the columns mn >= MN of a row, masked here,
  // and every k at or past the split's end (klim: a deep K-tile may overhang it).
  struct Fetch {
    int off[NV];   // byte offset at tile 0 (or -1: masked for every tile)
    int kpos[NV];  // the float4's k within a K-tile
  };
  __device__ __forceinline__ void fetch_init(Fetch& f, int64_t ld, int64_t mn0, int64_t mnlim,
                                             int64_t kbeg, int tid) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int mn, k;
      coords(tid + v * NT, mn, k);
      const int64_t gmn = mn0 + mn, gk = kbeg + k;
      const int64_t e = KC ? gmn * ld + gk : gk * ld + gmn;
      f.off[v] = (KC || gmn < mnlim) ? (int)(e * 4) : -1;
      f.kpos[v] = k;
    }
  }
  __device__ __forceinline__ void fetch4(int v, const Fetch& f, __amdgpu_buffer_rsrc_t rsrc,
                                         int tile_step, int t, int kt0, int klim) {
    const bool ok = f.off[v] >= 0 && kt0 + f.kpos[v] < klim;
    const int off = ok ? f.off[v] + t * tile_step : 0x7ffffff0;
    regs[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
  }

  // The same load for a stage wholly inside the split (no k test): the lane's tile-0 offset
  // (or a past-the-end one for a masked mn) in the VGPR, the stage's advance t * tile_step in
  // the scalar offset - no per-load VALU.
  __device__ __forceinline__ void fetch4s(int v, const Fetch& f, __amdgpu_buffer_rsrc_t rsrc,
                                          int soff) {
    const int off = f.off[v] >= 0 ? f.off[v] : 0x7ffffff0;
    regs[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, soff, 0));
  }

  // (!KC: a float4 is a 4-aligned mn run, which the bit-4 flip keeps contiguous)
  __device__ __forceinline__ void store_one(int v, float* __restrict__ lds, int tid) const {
    int mn, k;
    coords(tid + v * NT, mn, k);
    *reinterpret_cast<float4*>(lds + at(mn, k)) = regs[v];
  }

  __device__ __forceinline__ void store(float* __restrict__ lds, int tid) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) store_one(v, lds, tid);
  }

  // NS consecutive k-steps (k = kbase .. kbase+NS-1) of the 32-wide sub-tile at `off`
  // for this lane (row/col off + l32).
  template <int NS>
  __device__ __forceinline__ void frag(const float* __restrict__ lds, int off, int l32, int kbase,
                                       float (&f)[NS]) const {
    static_assert(NS % 4 == 0, "fragment length");
    if constexpr (KC) {
#pragma unroll
      for (int c = 0; c < NS / 4; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(lds + at(off + l32, kbase + 4 * c));
        f[4 * c + 0] = v.x;
        f[4 * c + 1] = v.y;
        f[4 * c + 2] = v.z;
        f[4 * c + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < NS; ++s) f[s] = lds[at(off + l32, kbase + s)];
    }
  }
};

// One scalar f32 add the SLP vectorizer cannot fuse into v_pk_add_f32 (a packed f32 op
// beside MFMAs costs ~26 cycles per MFMA gap on gfx950; a plain v_add_f32 is ~free).
__device__ __forceinline__ float add_f32(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // Contiguous block runs per XCD (blocks b and b+8 share an XCD); bijective for any nwg.
  const int xcd = bid % 8;
  const int q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// C = epilogue(v) where v = alpha * acc (already scaled); returns the value written.
__device__ __forceinline__ float apply_epilogue(const GemmParams& p, int64_t row, int64_t col,
                                                float v) {
  float* cp = p.C + row * p.ldc + col;
  switch (p.epi) {
    case DLRM_EPI_BIAS:
      v += p.bias[col];
      break;
    case DLRM_EPI_BIAS_RELU:
      v = fmaxf(v + p.bias[col], 0.f);
      break;
    case DLRM_EPI_RELU:
      v = fmaxf(v, 0.f);
      break;
    case DLRM_EPI_DRELU:
      v = p.aux[row * p.ldaux + col] > 0.f ? v : 0.f;
      break;
    case DLRM_EPI_SGD:
      v = *cp - v;
      break;
    case DLRM_EPI_ACCUM:
      v = *cp + v;
      break;
    default:
      break;
  }
  *cp = v;
  return v;
}

// The same epilogue for a compile-time kind, on values already loaded: old = the C element
// (SGD / ACCUM), aux = the mask operand (DRELU), bias = bias[col] (BIAS / BIAS_RELU).  The
// arithmetic is apply_epilogue's, so results are bitwise the same.
template <int EPI>
__device__ __forceinline__ float epi_value(float v, float old, float aux, float bias) {
  if constexpr (EPI == DLRM_EPI_BIAS) return v + bias;
  else if constexpr (EPI == DLRM_EPI_BIAS_RELU) return fmaxf(v + bias, 0.f);
  else if constexpr (EPI == DLRM_EPI_RELU) return fmaxf(v, 0.f);
  else if constexpr (EPI == DLRM_EPI_DRELU) return aux > 0.f ? v : 0.f;
  else if constexpr (EPI == DLRM_EPI_SGD) return old - v;
  else if constexpr (EPI == DLRM_EPI_ACCUM) return old + v;
  else return v;
}

__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void buf_st(float v, __amdgpu_buffer_rsrc_t r, int off) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, off, 0, 0);
}
constexpr int kOob = 0x7ffffff0;  // a byte offset past every descriptor (loads 0, stores dropped)

// The tile's epilogue for one kind, with no per-element branches and every operand load in
// flight at once: byte offsets from buffer descriptors over exactly the addressed extents,
// so rows past M land outside them (loads read 0, stores are dropped) and columns past N get
// kOob.  n elements at (row[q], col[q]) with values v[q] (already alpha-scaled).
template <int EPI, int NE>
__device__ __forceinline__ void store_elems(const GemmParams& p, const int (&row)[NE],
                                            const int (&col)[NE], const bool (&ok)[NE],
                                            const float (&v)[NE]) {
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.C, (short)0, (int)(((p.M - 1) * p.ldc + p.ldc) * 4), 0x00020000);
  int off[NE];
#pragma unroll
  for (int q = 0; q < NE; ++q)
    off[q] = ok[q] && row[q] < p.M ? (int)(((int64_t)row[q] * p.ldc + col[q]) * 4) : kOob;
  float old[NE], aux[NE], bias[NE];
#pragma unroll
  for (int q = 0; q < NE; ++q) old[q] = aux[q] = bias[q] = 0.f;
  if constexpr (EPI == DLRM_EPI_SGD || EPI == DLRM_EPI_ACCUM) {
#pragma unroll
    for (int q = 0; q < NE; ++q) old[q] = buf_ld(rc, off[q]);
  }
  if constexpr (EPI == DLRM_EPI_DRELU) {
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.aux, (short)0, (int)(((p.M - 1) * p.ldaux + p.ldaux) * 4), 0x00020000);
#pragma unroll
    for (int q = 0; q < NE; ++q)
      aux[q] = buf_ld(ra, ok[q] && row[q] < p.M ? (int)(((int64_t)row[q] * p.ldaux + col[q]) * 4)
                                                : kOob);
  }
  if constexpr (EPI == DLRM_EPI_BIAS || EPI == DLRM_EPI_BIAS_RELU) {
#pragma unroll
    for (int q = 0; q < NE; ++q) bias[q] = ok[q] ? p.bias[col[q]] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < NE; ++q) buf_st(epi_value<EPI>(v[q], old[q], aux[q], bias[q]), rc, off[q]);
}

// Offsets of C (and aux) fit the 32-bit buffer offsets with a tile of slack.
__device__ __forceinline__ bool epi_fits(const GemmParams& p) {
  const int64_t lim = 0x7ff00000LL;
  return (p.M + 256) * p.ldc * 4 < lim &&
         (p.epi != DLRM_EPI_DRELU || (p.M + 256) * p.ldaux * 4 < lim);
}

template <int NE>
__device__ __forceinline__ void store_elems_any(const GemmParams& p, const int (&row)[NE],
                                                const int (&col)[NE], const bool (&ok)[NE],
                                                const float (&v)[NE]) {
  switch (p.epi) {
    case DLRM_EPI_BIAS: return store_elems<DLRM_EPI_BIAS>(p, row, col, ok, v);
    case DLRM_EPI_BIAS_RELU: return store_elems<DLRM_EPI_BIAS_RELU>(p, row, col, ok, v);
    case DLRM_EPI_RELU: return store_elems<DLRM_EPI_RELU>(p, row, col, ok, v);
    case DLRM_EPI_DRELU: return store_elems<DLRM_EPI_DRELU>(p, row, col, ok, v);
    case DLRM_EPI_SGD: return store_elems<DLRM_EPI_SGD>(p, row, col, ok, v);
    case DLRM_EPI_ACCUM: return store_elems<DLRM_EPI_ACCUM>(p, row, col, ok, v);
    default: return store_elems<DLRM_EPI_STORE>(p, row, col, ok, v);
  }
}


// Split-K completion.  Each split workgroup stores its NV accumulators (fragment order,
// thread-major: rec[tid*NV + q]) and its row sums (rec[BM*BN + local row]) into its
// record, then takes a ticket; the last arriver sums every split's record in split order
// and applies the epilogue.  Publication across the (mutually non-coherent) per-XCD L2s is
// the write-through form of the MI355X guide: every record store and every record load is
// sc1, the stores are drained (s_waitcnt vmcnt(0)) and the workgroup synchronised before
// the agent-scope ticket; the last arriver resets the tile's ticket for the next launch.
// Returns true in the workgroup that must write the output (always when unsplit); v / rs
// then hold the full sums.
template <int BM, int BN, int NV, int FM>
__device__ __forceinline__ bool splitk_reduce(const GemmParams& p, int tile, int split,
                                              float (&v)[NV], float (&rs)[FM], int rs_row0,
                                              int rs_stride, bool rs_owner, float* smem) {
  if (p.splits <= 1) return true;
  constexpr int REC = BM * BN + BM;
  static_assert(NV % 4 == 0, "record chunks are float4");
  using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
  const int tid = threadIdx.x;
  float* tile_base = p.ws + (int64_t)tile * p.splits * REC;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)tile_base, (short)0, (int)(p.splits * REC * 4), 0x00020000);
#pragma unroll
  for (int q = 0; q < NV; q += 4) {
    const float4 f = make_float4(v[q], v[q + 1], v[q + 2], v[q + 3]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f), rr,
                                           (split * REC + tid * NV + q) * 4, 0, 16 /*sc1*/);
  }
  if (rs_owner) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, rs[i]), rr,
                                            (split * REC + BM * BN + rs_row0 + i * rs_stride) * 4,
                                            0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == p.splits - 1;
    if (last) __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    reinterpret_cast<volatile int*>(smem)[0] = last;
  }
  __syncthreads();
  if (!reinterpret_cast<volatile int*>(smem)[0]) return false;
  const int rrow = rs_owner ? rs_row0 : 0;  // every lane loads (valid address), owners use it
  auto load_rec = [&](int s, float4 (&t)[NV / 4], float (&tr)[FM]) {
    const int o = s * REC;
#pragma unroll
    for (int q = 0; q < NV / 4; ++q)
      t[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rr, (o + tid * NV + 4 * q) * 4, 0, 16));
#pragma unroll
    for (int i = 0; i < FM; ++i)
      tr[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            rr, (o + BM * BN + rrow + i * rs_stride) * 4, 0, 16));
  };
  auto add_rec = [&](const float4 (&t)[NV / 4], const float (&tr)[FM], bool first) {
#pragma unroll
    for (int q = 0; q < NV / 4; ++q) {
      v[4 * q + 0] = first ? t[q].x : v[4 * q + 0] + t[q].x;
      v[4 * q + 1] = first ? t[q].y : v[4 * q + 1] + t[q].y;
      v[4 * q + 2] = first ? t[q].z : v[4 * q + 2] + t[q].z;
      v[4 * q + 3] = first ? t[q].w : v[4 * q + 3] + t[q].w;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) rs[i] = first ? tr[i] : rs[i] + tr[i];
  };
  int s = 0;
  for (; s + 1 < p.splits; s += 2) {
    float4 t0[NV / 4], t1[NV / 4];
    float r0[FM], r1[FM];
    load_rec(s, t0, r0);
    load_rec(s + 1, t1, r1);
    add_rec(t0, r0, s == 0);
    add_rec(t1, r1, false);
  }
  if (s < p.splits) {
    float4 t0[NV / 4];
    float r0[FM];
    load_rec(s, t0, r0);
    add_rec(t0, r0, s == 0);
  }
  return true;
}

// Tile epilogue: PARTIAL slabs, or the split-K
// hand-off then the fused epilogue.  acc is the wave's FM x FN grid of 16x16 accumulators
// (register r: row 4*(lane>>4) + r, col lane&15 - the same map for every 16x16 MFMA form);
// rs[i] is the full (this split's) row sum of row wm0 + 16 i + (lane&15) of op(A).
template <int BM, int BN, int WGM, int WGN, bool RS, int FM, int FN>
__device__ __forceinline__ void finish_tile(const GemmParams& p, const f32x4 (&acc)[FM][FN],
                                            float (&rs)[FM], int tile, int split, int tn,
                                            int64_t m0, int64_t n0, float* smem) {
  constexpr int WM = BM / WGM, WN = BN / WGN;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int kq = lane >> 4;
  const int l16 = lane & 15;
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;
  // Owners of the row sums: kq == 0 lanes of the left wave column, first column of tiles.
  const bool rs_owner = RS && tn == 0 && (wave % WGN) == 0 && kq == 0;

  constexpr int NV = FM * FN * 4;
  float v[NV];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[(i * FN + j) * 4 + r] = acc[i][j][r];
  if (p.mode == DLRM_GEMM_PARTIAL && p.M * p.N * 4 < 0x7ff00000LL) {
    // raw partial sums for a REDUCE job of a later launch (the kernel boundary publishes),
    // as buffer stores from one descriptor per slab: no per-element branch or 64-bit address
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.part + (int64_t)split * p.M * p.N), (short)0, (int)(p.M * p.N * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = (int)(n0 + wn0 + j * 16 + l16);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = (int)(m0 + wm0 + i * 16 + 4 * kq + r);
          buf_st(v[(i * FN + j) * 4 + r], rp,
                 row < p.M && col < p.N ? (int)(((int64_t)row * p.N + col) * 4) : kOob);
        }
      }
    if (rs_owner) {
      float* rslab = p.part + (int64_t)p.splits * p.M * p.N + (int64_t)split * p.M;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int64_t row = m0 + wm0 + i * 16 + l16;
        if (row < p.M) rslab[row] = rs[i];
      }
    }
    return;
  }
  if (p.mode == DLRM_GEMM_PARTIAL) {
    // raw partial sums for a REDUCE job of a later launch (the kernel boundary publishes)
    float* slab = p.part + (int64_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t col = n0 + wn0 + j * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = m0 + wm0 + i * 16 + 4 * kq + r;
          if (row < p.M && col < p.N) slab[row * p.N + col] = v[(i * FN + j) * 4 + r];
        }
      }
    if (rs_owner) {
      float* rslab = p.part + (int64_t)p.splits * p.M * p.N + (int64_t)split * p.M;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int64_t row = m0 + wm0 + i * 16 + l16;
        if (row < p.M) rslab[row] = rs[i];
      }
    }
    return;
  }
  if (!splitk_reduce<BM, BN, NV, FM>(p, tile, split, v, rs, wm0 + l16, 16, rs_owner, smem))
    return;
  if (epi_fits(p)) {  // batched: every operand load in flight at once, no per-element branch
    int row[NV], col[NV];
    bool ok[NV];
    float w[NV];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = (i * FN + j) * 4 + r;
          row[q] = (int)(m0 + wm0 + i * 16 + 4 * kq + r);
          col[q] = (int)(n0 + wn0 + j * 16 + l16);
          ok[q] = col[q] < p.N;
          w[q] = __fmul_rn(p.alpha, v[q]);  // rounded alone, as apply_epilogue sees it
        }
    store_elems_any<NV>(p, row, col, ok, w);
    if constexpr (RS) {
      int rrow[FM], rcol[FM];
      bool rok[FM];
      float rw[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        rrow[i] = (int)(m0 + wm0 + i * 16 + l16);
        rcol[i] = (int)p.ones_col;
        rok[i] = rs_owner;
        rw[i] = __fmul_rn(p.alpha, rs[i]);
      }
      store_elems_any<FM>(p, rrow, rcol, rok, rw);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = n0 + wn0 + j * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm0 + i * 16 + 4 * kq + r;
        if (row < p.M && col < p.N) apply_epilogue(p, row, col, p.alpha * v[(i * FN + j) * 4 + r]);
      }
    }
  if (rs_owner) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int64_t row = m0 + wm0 + i * 16 + l16;
      if (row < p.M) apply_epilogue(p, row, p.ones_col, p.alpha * rs[i]);
    }
  }
}


// One output tile (and K split) of problem p: the software-pipelined 16x16x4 body.  The
// workgroup is WGM x WGN waves, each owning a (BM/WGM) x (BN/WGN) sub-tile.  A K-tile (one
// LDS stage, one barrier) is U sub-tiles of 32: deeper stages (U = 2, 4) halve or quarter
// the barriers and read the next sub-tile's fragments from the SAME buffer during the
// current one's MFMAs.  The MFMA sequence over k is the U = 1 sequence for every U (sub-tile
// after sub-tile, the same k-quarter permutation inside each): results are bitwise those of
// U = 1 (a stage overhanging the split's end multiplies zeros).
template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, bool RS, int U = 1>
__device__ __forceinline__ void pipe_body(const GemmParams& p, int lb, float* smem) {
  static_assert(U == 1 || U % 2 == 0, "sub-tiles per stage: 1 or even");
  constexpr int NT = WGM * WGN * 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile");
  constexpr int KL = kBK / 4;  // k-steps per 32-deep sub-tile (a lane group owns KL consecutive k)
  constexpr int BKT = kBK * U;  // k per LDS stage
  using SA = Stage<BM, BKT, A_KC, true, NT, true>;
  using SB = Stage<BN, BKT, B_KC, true, NT, true>;
  constexpr int NS = SA::NV + SB::NV;  // staged float4 per thread per stage
  static_assert(NS <= U * KL - 1, "staging must finish before the barrier step");

  const int tile = lb / p.splits;
  const int split = lb - tile * p.splits;
  // Grouped raster: runs of kRasterRows tile rows are walked column by column, so the
  // contiguous run of tiles an XCD receives (xcd_remap) is a 2-D block - a few hundred rows
  // of each operand in its 4 MiB L2 instead of a band of A rows against ALL of B.  A
  // bijection on the tiles (the tail group takes the rows left); the sums are unchanged.
  int tm, tn;
  {
    constexpr int G = kRasterRows;
    const int per_group = G * p.tiles_n;
    const int grp = tile / per_group, first = grp * G;
    const int gsz = p.tiles_m - first < G ? p.tiles_m - first : G;
    const int pos = tile - grp * per_group;
    tm = first + pos % gsz;
    tn = pos / gsz;
  }
  if constexpr (RS) {
    // only the first column of tiles owns the row sums (finish_tile): the others run the
    // body without the per-k-step adds (one VALU per MFMA)
    if (tn != 0) return pipe_body<BM, BN, WGM, WGN, A_KC, B_KC, false, U>(p, lb, smem);
  }
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int kq = lane >> 4;
  const int l16 = lane & 15;
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rs[FM];  // row sums of op(A) over this lane's k (ones_col)
#pragma unroll
  for (int i = 0; i < FM; ++i) rs[i] = 0.f;

  const int nsub = (int)((kend - kbeg + kBK - 1) / kBK);
  const int nk = (nsub + U - 1) / U;
  SA sa;
  SB sb;
  // buffer descriptors over exactly the addressed extent (host guarantees < 2 GiB)
  const int64_t a_ext = A_KC ? (p.M - 1) * p.lda + p.K : (p.K - 1) * p.lda + p.M;
  const int64_t b_ext = B_KC ? (p.N - 1) * p.ldb + p.K : (p.K - 1) * p.ldb + p.N;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)(a_ext * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)(b_ext * 4), 0x00020000);
  typename SA::Fetch fa;
  typename SB::Fetch fb;
  sa.fetch_init(fa, p.lda, m0, p.M, kbeg, tid);
  sb.fetch_init(fb, p.ldb, n0, p.N, kbeg, tid);
  const int a_step = A_KC ? BKT * 4 : (int)(BKT * p.lda * 4);
  const int b_step = B_KC ? BKT * 4 : (int)(BKT * p.ldb * 4);
  const int kb32 = (int)kbeg, kend32 = (int)kend;
  auto fetch_one = [&](int c, int t) {  // staged float4 c of stage t (zeros past the split)
    if (c < SA::NV)
      sa.fetch4(c, fa, ra, a_step, t, kb32 + t * BKT, kend32);
    else
      sb.fetch4(c - SA::NV, fb, rb, b_step, t, kb32 + t * BKT, kend32);
  };
  // fast: stage t lies wholly inside the split (uniform; see Stage::fetch4s)
  auto fetch_any = [&](int c, int t, auto fast) {
    if constexpr (decltype(fast)::value) {
      if (c < SA::NV)
        sa.fetch4s(c, fa, ra, t * a_step);
      else
        sb.fetch4s(c - SA::NV, fb, rb, t * b_step);
    } else {
      fetch_one(c, t);
    }
  };
  auto put_one = [&](int c, float* buf) {
    if (c < SA::NV)
      sa.store_one(c, buf, tid);
    else
      sb.store_one(c - SA::NV, buf + SA::SIZE, tid);
  };
  auto read_frags = [&](const float* buf, int u, float (&a)[FM][KL], float (&b)[FN][KL]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
      sa.template frag<KL>(buf, wm0 + i * 16, l16, u * kBK + kq * KL, a[i]);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      sb.template frag<KL>(buf + SA::SIZE, wn0 + j * 16, l16, u * kBK + kq * KL, b[j]);
  };
  auto mfma_step = [&](float (&ca)[FM][KL], float (&cb)[FN][KL], int s) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[i][s], cb[j][s], acc[i][j], 0, 0, 0);
    if constexpr (RS) {
#pragma unroll
      for (int i = 0; i < FM; ++i) rs[i] = add_f32(rs[i], ca[i][s]);
    }
  };

  float a[FM][KL], b[FN][KL];
  // Prologue: stage 0 -> LDS buffer 0, stage 1 staged in registers, sub-tile 0 fragments
  // read.  Every fetch is unconditional: stages past nk load zeros (never used).
  DLRM_GEMM_STAMP(0);
  {
    // stage 1's loads are issued into a second register set before stage 0 is waited for,
    // so the two cold-cache round trips of the prologue overlap; stage 1 then moves to the
    // set the loop stages from
    SA sa1;
    SB sb1;
#pragma unroll
    for (int c = 0; c < NS; ++c) fetch_one(c, 0);
#pragma unroll
    for (int c = 0; c < SA::NV; ++c) sa1.fetch4(c, fa, ra, a_step, 1, kb32 + BKT, kend32);
#pragma unroll
    for (int c = 0; c < SB::NV; ++c) sb1.fetch4(c, fb, rb, b_step, 1, kb32 + BKT, kend32);
#pragma unroll
    for (int c = 0; c < NS; ++c) put_one(c, smem);
#pragma unroll
    for (int c = 0; c < SA::NV; ++c) sa.regs[c] = sa1.regs[c];
#pragma unroll
    for (int c = 0; c < SB::NV; ++c) sb.regs[c] = sb1.regs[c];
  }
  __syncthreads();
  read_frags(smem, 0, a, b);
  DLRM_GEMM_STAMP(1);

  // Sub-tile u of stage kt: MFMAs on (ca, cb) with the staging of stage kt+1 / fetch of kt+2
  // interleaved (staged float4 g = u*KL + step); a non-final sub-tile first issues the reads
  // of sub-tile u+1 into (na, nb) from the same buffer; the final one ends with the barrier
  // and sub-tile 0 of stage kt+1 read under its last k-step.
  auto subtile = [&](int kt, int u, float (&ca)[FM][KL], float (&cb)[FN][KL],
                     float (&na)[FM][KL], float (&nb)[FN][KL], auto fast) {
    const float* cur = smem + (kt & 1) * (SA::SIZE + SB::SIZE);
    float* nbuf = smem + ((kt + 1) & 1) * (SA::SIZE + SB::SIZE);
    const bool last = u == U - 1;
    if (!last) read_frags(cur, u + 1, na, nb);
#pragma unroll
    for (int s = 0; s < KL - 1; ++s) {
      mfma_step(ca, cb, s);
      const int g = u * KL + s;
      if (g < NS) {
        put_one(g, nbuf);            // stage t+1 (staged last stage) -> LDS
        fetch_any(g, kt + 2, fast);  // refill the register with stage t+2
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the interleave: no hoisting across steps
    }
    if (!last) {
      mfma_step(ca, cb, KL - 1);
      const int g = u * KL + KL - 1;
      if (g < NS) {
        put_one(g, nbuf);
        fetch_any(g, kt + 2, fast);
      }
      __builtin_amdgcn_sched_barrier(0);
    } else {
      __syncthreads();  // stage t+1 is complete in LDS
      read_frags(nbuf, 0, na, nb);
      __builtin_amdgcn_sched_barrier(0);  // issue the reads before the last step's MFMAs
      mfma_step(ca, cb, KL - 1);
    }
  };
  float a1[FM][KL], b1[FN][KL];
  if constexpr (U == 1) {  // fragment sets ping-pong across stages: unrolled by two
    // the fetches of sub-tile kt are stage kt + 2's: wholly inside the split while
    // kbeg + (kt + 3) * BKT <= kend (then no per-load k test)
    const std::true_type fast{};
    const std::false_type slow{};
    for (int kt = 0; kt < nk; kt += 2) {
      if (kb32 + (kt + 3) * BKT <= kend32)
        subtile(kt, 0, a, b, a1, b1, fast);
      else
        subtile(kt, 0, a, b, a1, b1, slow);
      DLRM_GEMM_STAMP(2 + kt);
      if (kt + 1 >= nk) break;
      if (kb32 + (kt + 4) * BKT <= kend32)
        subtile(kt + 1, 0, a1, b1, a, b, fast);
      else
        subtile(kt + 1, 0, a1, b1, a, b, slow);
      DLRM_GEMM_STAMP(3 + kt);
    }
  } else {  // an even number of sub-tiles per stage: every stage starts on (a, b)
    for (int kt = 0; kt < nk; ++kt) {
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        subtile(kt, u, a, b, a1, b1, std::false_type{});
        subtile(kt, u + 1, a1, b1, a, b, std::false_type{});
      }
    }
  }

  // Row sums: lanes l16, l16+16, l16+32, l16+48 hold the four k-quarters of row l16
  // (fixed pairing order: deterministic).
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
  }
  DLRM_GEMM_STAMP(-2);
  finish_tile<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0, smem);
  DLRM_GEMM_STAMP(-1);
}

// REDUCE job: C = epi(alpha * sum_s part[s]) in split order (the same additions as the
// in-launch reduction), one float4 of the [M][N] slab per thread, then one row sum per
// thread for ones_col.  Up to 8 splits' loads in flight.
__device__ __forceinline__ void reduce_body(const GemmParams& p, int lb) {
  const int64_t MN = p.M * p.N;
  const int64_t i = (int64_t)lb * blockDim.x + threadIdx.x;
  const int64_t n4 = MN / 4;  // N % 4 == 0 (host check)
  const int S = p.splits;
  if (i < n4) {
    const float4* src = reinterpret_cast<const float4*>(p.part) + i;
    const int64_t stride = MN / 4;
    float4 acc = src[0];
    for (int s0 = 1; s0 < S; s0 += 8) {
      float4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (s0 + u < S) t[u] = src[(int64_t)(s0 + u) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (s0 + u < S) {
          acc.x += t[u].x;
          acc.y += t[u].y;
          acc.z += t[u].z;
          acc.w += t[u].w;
        }
    }
    const int64_t e = 4 * i, row = e / p.N, col = e - row * p.N;
    if (p.epi == DLRM_EPI_SGD || p.epi == DLRM_EPI_ACCUM) {
      // the four old values loaded together (the generic path waits for each in turn)
      float* cp = p.C + row * p.ldc + col;
      const float o0 = cp[0], o1 = cp[1], o2 = cp[2], o3 = cp[3];
      const bool sgd = p.epi == DLRM_EPI_SGD;
      // alpha * acc rounded on its own (no contraction into the add): apply_epilogue's
      // arithmetic, bitwise
      const float v0 = __fmul_rn(p.alpha, acc.x), v1 = __fmul_rn(p.alpha, acc.y);
      const float v2 = __fmul_rn(p.alpha, acc.z), v3 = __fmul_rn(p.alpha, acc.w);
      cp[0] = sgd ? o0 - v0 : o0 + v0;
      cp[1] = sgd ? o1 - v1 : o1 + v1;
      cp[2] = sgd ? o2 - v2 : o2 + v2;
      cp[3] = sgd ? o3 - v3 : o3 + v3;
      return;
    }
    apply_epilogue(p, row, col, p.alpha * acc.x);
    apply_epilogue(p, row, col + 1, p.alpha * acc.y);
    apply_epilogue(p, row, col + 2, p.alpha * acc.z);
    apply_epilogue(p, row, col + 3, p.alpha * acc.w);
  } else if (p.ones_col >= 0 && i - n4 < p.M) {
    const int64_t row = i - n4;
    const float* rsrc = p.part + (int64_t)S * MN + row;
    float acc = rsrc[0];
    for (int s = 1; s < S; ++s) acc += rsrc[(int64_t)s * p.M];
    apply_epilogue(p, row, p.ones_col, p.alpha * acc);
  }
}

template <int BM, int BN, int U = 1>
constexpr int group_smem_floats() {
  // double-buffered A and B panels of U 32-deep sub-tiles (unpadded swizzled images: the
  // same size for every operand layout)
  return 2 * (BM + BN) * kBK * U;
}

// Body kinds: the four operand layouts, plus 4 = layout 2 (wgrad) with the row sums.
__host__ __device__ constexpr int kind_bit(int layout, bool rs) { return 1 << (rs ? 4 : layout); }

// Up to kMaxGroup independent problems; block -> (problem, tile, split) after the XCD remap.
// KINDS is the set of body kinds compiled in (a launch uses the smallest instantiation that
// covers its problems: fewer bodies, fewer registers).
template <int BM, int BN, int WGM, int WGN, int KINDS, int U = 1>
__device__ __forceinline__ void group_body(const GemmGroup& g, int b, float* smem) {
  // Problems own consecutive PHYSICAL block ranges, so each one is dealt round-robin over
  // all eight XCDs (a remap across the whole launch would give each problem a few XCDs);
  // inside its range the XCD remap gives each XCD a contiguous run of that problem's tiles.
  int q = 0;
#pragma unroll
  for (int i = 1; i < kMaxGroup; ++i)
    if (i < g.n && b >= g.p[i].block0) q = i;
  const GemmParams& p = g.p[q];
  const int nq = (q + 1 < g.n ? g.p[q + 1].block0 : g.total) - p.block0;
  const int lb = xcd_remap(b - p.block0, nq);
  if (p.mode == DLRM_GEMM_REDUCE) return reduce_body(p, lb);
  const int kind = (p.layout == 2 && p.ones_col >= 0) ? 4 : p.layout;
  if constexpr ((KINDS & 1) != 0)
    if (kind == 0) return pipe_body<BM, BN, WGM, WGN, true, true, false, U>(p, lb, smem);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return pipe_body<BM, BN, WGM, WGN, true, false, false, U>(p, lb, smem);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return pipe_body<BM, BN, WGM, WGN, false, false, false, U>(p, lb, smem);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return pipe_body<BM, BN, WGM, WGN, false, true, false, U>(p, lb, smem);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return pipe_body<BM, BN, WGM, WGN, false, false, true, U>(p, lb, smem);
}

template <int BM, int BN, int WGM, int WGN, int KINDS, int U = 1>
__global__ __launch_bounds__(WGM * WGN * 64, 2) void gemm_group_kernel(
    const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN, U>()];
  group_body<BM, BN, WGM, WGN, KINDS, U>(g, blockIdx.x, smem);
}

// The group plus one pass of a deferred embedding update (tbe_bwd_roles.hpp) in the same
// launch: workgroups [0, r.blocks) run the pass (dispatched first: its HBM-latency-bound
// waves start before the GEMM tiles fill the CUs), the rest the GEMM problems.  Tiles
// 64x32 / 32x64 only, at >= 4 waves per SIMD (<= 128 VGPRs: the pass alone would take
// twice that, and the GEMM tiles would run at half their occupancy).
template <int BM, int BN, int WGM, int WGN, int PHASE>
__global__ __launch_bounds__(WGM * WGN * 64, 4) void gemm_role_kernel(const GemmGroup g,
                                                                      const LaunchRole r) {
  __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN>()];
  const int b = blockIdx.x;
  if (b < r.blocks) return tbe_role_run<PHASE>(r, b, smem);
  group_body<BM, BN, WGM, WGN, 31>(g, b - r.blocks, smem);
}

// Fallback for operands the pipelined body cannot take (unaligned rows, ragged float4
// extents, > 2 GiB extents): 32x32x2 MFMA, register-staged, unsplit, element-guarded.
template <bool A_KC, bool B_KC>
__global__ __launch_bounds__(kThreads, 2) void gemm_generic_kernel(const GemmParams p) {
  constexpr int BM = 64, BN = 64, BKT = 32;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int NSTEP = BKT / 2;  // MFMA k-steps per wave per K-tile
  using SA = Stage<BM, BKT, A_KC, false, kThreads>;
  using SB = Stage<BN, BKT, B_KC, false, kThreads>;
  __shared__ __attribute__((aligned(16))) float smem[2 * (SA::SIZE + SB::SIZE)];
  float* As0 = smem;
  float* Bs0 = smem + SA::SIZE;
  float* As1 = smem + SA::SIZE + SB::SIZE;
  float* Bs1 = As1 + SA::SIZE;
  const int tile = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
  const int tm = tile / p.tiles_n, tn = tile - (tile / p.tiles_n) * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int h = lane >> 5, l32 = lane & 31;
  const int wm0 = (wave >> 1) * WM, wn0 = (wave & 1) * WN;
  f32x16 acc, acc2;  // two chains alternate over the k-steps (64-cycle accumulate latency)
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
  SA sa;
  SB sb;
  const int64_t nk = (p.K + BKT - 1) / BKT;
  if (nk > 0) {
    sa.load(p.A, p.lda, m0, p.M, 0, p.K, tid);
    sb.load(p.B, p.ldb, n0, p.N, 0, p.K, tid);
    sa.store(As0, tid);
    sb.store(Bs0, tid);
  }
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const bool odd = kt & 1;
    const float* As = odd ? As1 : As0;
    const float* Bs = odd ? Bs1 : Bs0;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(p.A, p.lda, m0, p.M, (kt + 1) * BKT, p.K, tid);
      sb.load(p.B, p.ldb, n0, p.N, (kt + 1) * BKT, p.K, tid);
    }
    float a[NSTEP], b[NSTEP];
    sa.template frag<NSTEP>(As, wm0, l32, h * NSTEP, a);
    sb.template frag<NSTEP>(Bs, wn0, l32, h * NSTEP, b);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      if (s & 1)
        acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc2, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
    }
    if (more) {
      sa.store(odd ? As0 : As1, tid);
      sb.store(odd ? Bs0 : Bs1, tid);
    }
    __syncthreads();
  }
  acc += acc2;
  // accumulator register r of a 32x32 tile: row (r&3) + 8*(r>>2) + 4*(lane>>5), col lane&31
  const int64_t col = n0 + wn0 + l32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = m0 + wm0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < p.M && col < p.N) apply_epilogue(p, row, col, p.alpha * acc[r]);
  }
}

// Fallback row sum (ones_col for the generic kernel): C[m][ones_col] =
// epi(alpha * sum_k op(A)(m, k)); 64 rows x 4 k-slices per block, slices added in order.
__global__ __launch_bounds__(kThreads) void gemm_rowsum_kernel(const GemmParams p, bool a_kc) {
  __shared__ float part[4][64];
  const int tid = threadIdx.x, r = tid & 63, ks = tid >> 6;
  const int64_t m = (int64_t)blockIdx.x * 64 + r;
  float s = 0.f;
  if (m < p.M)
    for (int64_t k = ks; k < p.K; k += 4) s += a_kc ? p.A[m * p.lda + k] : p.A[k * p.lda + m];
  part[ks][r] = s;
  __syncthreads();
  if (ks == 0 && m < p.M)
    apply_epilogue(p, m, p.ones_col, p.alpha * (((part[0][r] + part[1][r]) + part[2][r]) + part[3][r]));
}

// ------------------------------------------------------------------- planning --
struct Plan {
  int splits = 1;
  int64_t kchunk = 0;
};

Plan make_plan(int64_t s, int64_t K) {
  if (s > kMaxSplit) s = kMaxSplit;
  int64_t smax = dlrm::ceil_div(K, kBK);
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  int64_t kchunk = dlrm::ceil_div(dlrm::ceil_div(K, s), kBK) * kBK;
  if (kchunk < kBK) kchunk = kBK;
  Plan pl;
  pl.splits = (int)dlrm::ceil_div(K, kchunk);
  pl.kchunk = kchunk;
  return pl;
}

struct Desc {  // one problem as the host sees it
  int32_t trans_a, trans_b;
  int64_t M, N, K;
  float alpha;
  const float *A, *B;
  int64_t lda, ldb;
  float* C;
  int64_t ldc;
  int32_t epi;
  const float* bias;
  const float* aux;
  int64_t ldaux;
  int64_t ones_col;
  int32_t mode = DLRM_GEMM_FULL;
  int32_t splits = 0;
  float* part = nullptr;
};

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// The pipelined body moves whole float4s through 32-bit buffer offsets.
bool pipe_ok(const Desc& d) {
  const bool a_kc = !d.trans_a, b_kc = d.trans_b != 0;
  const int64_t a_ext = a_kc ? (d.M - 1) * d.lda + d.K : (d.K - 1) * d.lda + d.M;
  const int64_t b_ext = b_kc ? (d.N - 1) * d.ldb + d.K : (d.K - 1) * d.ldb + d.N;
  return aligned16(d.A) && aligned16(d.B) && d.lda % 4 == 0 && d.ldb % 4 == 0 && d.K % 4 == 0 &&
         (a_kc || d.M % 4 == 0) && (b_kc || d.N % 4 == 0) && a_ext * 4 < 0x7ff00000LL &&
         b_ext * 4 < 0x7ff00000LL;
}

int layout_of(const Desc& d) {
  const bool a_kc = !d.trans_a, b_kc = d.trans_b != 0;
  return a_kc ? (b_kc ? 0 : 1) : (b_kc ? 3 : 2);
}

struct PlanEntry {
  int64_t M, N, K;
  int layout, bm, bn, split;
  int wm = 2, wn = 2;
};

// Measured plans for the DLRM step shapes of single-problem launches (exact match), from
// tools/gemm_sweep.py on MI355X.
constexpr PlanEntry kPlans[] = {
#include "gemm_plans.inc"
    {0, 0, 0, 0, 64, 64, 1},  // sentinel (never matches: M = 0)
};

// Compiled tiles (BM x BN on 2x2 waves): 64x64, 128x64, 64x128, 32x64, 64x32, 32x32 (the
// latency-bound small-batch shapes: twice the workgroups of 64x32 without a K split,
// profiles/r05_gemm_plans_resweep.txt).  (Other
// wave layouts of pipe_body - 64x32 on 2x1, 32x64 on 1x2, 128x32 on 4x1 - measured slower
// on every DLRM shape: tools/gemm_cfg_ab.py, profiles/r02_gemm_cfg_ab.txt.)
// (Deep LDS stages - pipe_body U = 2 / 4, two or four 32-deep sub-tiles per barrier - are
// bitwise the same and measured slower at every tile on every C3 shape:
// profiles/r06_gemm_deep_stage_lab.txt.  The product compiles U = 1 only.)
bool tile_ok(int bm, int bn, int wm, int wn) {
  return wm == 2 && wn == 2 &&
         ((bm == 64 && bn == 64) || (bm == 128 && bn == 64) || (bm == 64 && bn == 128) ||
          (bm == 32 && bn == 64) || (bm == 64 && bn == 32) || (bm == 32 && bn == 32));
}

struct Tile {
  int bm = 64, bn = 32, wm = 2, wn = 2;
  bool operator==(const Tile& o) const {
    return bm == o.bm && bn == o.bn && wm == o.wm && wn == o.wn;
  }
};

// Plan of ONE problem, independent of what it is grouped with (so a problem's result is
// bitwise the same in any group: the split decides the summation order, the tile shape
// does not).
void plan_one(const Desc& d, Tile& t, Plan& pl) {
  t = Tile{64, 64, 2, 2};
  if (d.mode == DLRM_GEMM_REDUCE) {  // elementwise job: no tiles, no K
    pl.splits = d.splits;
    pl.kchunk = 0;
    return;
  }
  if (d.mode == DLRM_GEMM_PARTIAL && d.splits > 0) {  // caller-sized partial buffer
    Desc q = d;
    q.mode = DLRM_GEMM_FULL;
    plan_one(q, t, pl);
    pl = make_plan(d.splits, d.K);
    return;
  }
  // plan overrides (dlrm_set_tuning; sweeps and coverage tests)
  if (const int64_t tile = dlrm::tuning(DLRM_TUNE_GEMM_TILE)) {
    const int a = (int)(tile / 1000), b = (int)(tile % 1000);
    if (tile_ok(a, b, 2, 2)) t = Tile{a, b, 2, 2};
    const int64_t fs = dlrm::tuning(DLRM_TUNE_GEMM_SPLIT);
    pl = make_plan(fs > 0 ? fs : 1, d.K);
    return;
  }
  const bool use_table = true;
  if (use_table)
    for (const PlanEntry& e : kPlans)
      if (e.M == d.M && e.N == d.N && e.K == d.K && e.layout == layout_of(d)) {
        t = Tile{e.bm, e.bn, e.wm, e.wn};
        pl = make_plan(e.split, d.K);
        return;
      }
  // Heuristic (shapes not in the table): 64x32 tiles (the sweep's best almost everywhere);
  // FULL problems run unsplit unless they have fewer than one tile per CU (an in-launch
  // split costs a hand-off); PARTIAL ones split K until >= 2 blocks per CU, every K chunk
  // >= 256 (8 K-tiles).
  t = Tile{64, 32, 2, 2};
  const int64_t tiles = dlrm::ceil_div(d.M, 64) * dlrm::ceil_div(d.N, 32);
  const int target = d.mode == DLRM_GEMM_PARTIAL ? 512 : 256;
  int64_t s = 1;
  while (tiles * s < target && dlrm::ceil_div(d.K, s + 1) >= 256 && s < kMaxSplit) ++s;
  pl = make_plan(s, d.K);
}

// Tile config of a launch: the GEMM problems' common choice, else 64x32 (REDUCE jobs have
// no tiles and do not vote).
void plan_launch(int n, const Desc* d, Tile& t, Plan* pl) {
  bool first = true;
  t = Tile{64, 64, 2, 2};
  for (int i = 0; i < n; ++i) {
    Tile a;
    plan_one(d[i], a, pl[i]);
    if (d[i].mode == DLRM_GEMM_REDUCE) continue;
    if (first) {
      t = a;
      first = false;
    } else if (!(a == t)) {
      t = Tile{64, 32, 2, 2};
    }
  }
  if (t.bm == 128 && t.bn == 128) t = Tile{64, 32, 2, 2};
}

// Split-K tickets (tiles of in-launch split problems) a launch on tile t needs.
int64_t split_tiles(int n, const Desc* d, const Tile& t, const Plan* pl) {
  int64_t tick = 0;
  for (int i = 0; i < n; ++i)
    if (pl[i].splits > 1 && d[i].mode == DLRM_GEMM_FULL)
      tick += dlrm::ceil_div(d[i].M, t.bm) * dlrm::ceil_div(d[i].N, t.bn);
  return tick;
}

// Split-K workspace: the fixed 64 KiB ticket head, then each problem's records.
size_t group_ws_bytes(int n, const Desc* d, const Tile& t, const Plan* pl) {
  const int bm = t.bm, bn = t.bn;
  WsCarver c(nullptr);
  c.take<int>(kTicketCap);
  bool any = false;
  for (int i = 0; i < n; ++i)
    if (pl[i].splits > 1 && d[i].mode == DLRM_GEMM_FULL) {
      any = true;
      const int64_t tiles = dlrm::ceil_div(d[i].M, bm) * dlrm::ceil_div(d[i].N, bn);
      c.take<float>((size_t)tiles * pl[i].splits * (bm * bn + bm));
    }
  return any ? c.used + 256 : 0;
}

template <int BM, int BN, int U = 1, int WGM = 2, int WGN = 2>
int launch_group(int n, const Desc* d, const Plan* pl, void* ws, size_t ws_bytes,
                 const LaunchRole* role, int phase, hipStream_t st) {
  constexpr int NT = WGM * WGN * 64;
  GemmGroup g{};
  g.n = n;
  WsCarver c(ws);
  int* tickets = c.take<int>(kTicketCap);
  int64_t tick = 0, blocks = 0;
  for (int i = 0; i < n; ++i) {
    GemmParams& p = g.p[i];
    p.M = d[i].M, p.N = d[i].N, p.K = d[i].K, p.alpha = d[i].alpha;
    p.A = d[i].A, p.lda = d[i].lda, p.B = d[i].B, p.ldb = d[i].ldb;
    p.C = d[i].C, p.ldc = d[i].ldc, p.epi = d[i].epi, p.bias = d[i].bias;
    p.aux = d[i].aux, p.ldaux = d[i].ldaux, p.ones_col = d[i].ones_col;
    p.layout = layout_of(d[i]);
    p.mode = d[i].mode;
    p.part = d[i].part;
    p.tiles_m = (int)dlrm::ceil_div(p.M, BM);
    p.tiles_n = (int)dlrm::ceil_div(p.N, BN);
    p.splits = pl[i].splits;
    p.kchunk = pl[i].kchunk > 0 ? pl[i].kchunk : kBK;
    p.block0 = (int)blocks;
    if (p.mode == DLRM_GEMM_REDUCE) {
      blocks += dlrm::ceil_div(p.M * p.N / 4 + (p.ones_col >= 0 ? p.M : 0), NT);
      continue;
    }
    if (p.splits > 1 && p.mode == DLRM_GEMM_FULL) {
      const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n;
      p.counters = tickets + tick;
      p.ws = c.take<float>((size_t)tiles * p.splits * (BM * BN + BM));
      tick += tiles;
    }
    blocks += (int64_t)p.tiles_m * p.tiles_n * p.splits;
  }
  DLRM_REQUIRE(tick <= kTicketCap && blocks < INT32_MAX, DLRM_ERR_UNSUPPORTED,
               "dlrm_gemm_f32: too many split tiles in one launch");
  DLRM_REQUIRE(tick == 0 || (ws && ws_bytes >= c.used), DLRM_ERR_WORKSPACE,
               "dlrm_gemm_f32: workspace too small");
  g.total = (int)blocks;
  int kinds = 0;
  for (int i = 0; i < n; ++i)
    if (g.p[i].mode != DLRM_GEMM_REDUCE)
      kinds |= kind_bit(g.p[i].layout, g.p[i].layout == 2 && g.p[i].ones_col >= 0);
  if constexpr (U == 1 && ((BM == 64 && BN == 32) || (BM == 32 && BN == 64))) {
    if (role) {  // + a deferred embedding-update pass (every body kind compiled in)
      static_assert(NT == 256, "the update passes run 256-thread workgroups");
      DLRM_REQUIRE((int64_t)role->blocks + blocks < INT32_MAX, DLRM_ERR_UNSUPPORTED,
                   "dlrm_gemm_f32_group_role: too many workgroups");
      const dim3 grid(role->blocks + g.total), block(NT);
      if (phase == 1)
        hipLaunchKernelGGL((gemm_role_kernel<BM, BN, WGM, WGN, 1>), grid, block, 0, st, g, *role);
      else if (phase == 2)
        hipLaunchKernelGGL((gemm_role_kernel<BM, BN, WGM, WGN, 2>), grid, block, 0, st, g, *role);
      else
        hipLaunchKernelGGL((gemm_role_kernel<BM, BN, WGM, WGN, 4>), grid, block, 0, st, g, *role);
      DLRM_LAUNCH_CHECK("dlrm_gemm_f32_group_role");
      return DLRM_OK;
    }
  } else {
    DLRM_REQUIRE(!role, DLRM_ERR_UNSUPPORTED, "dlrm_gemm_f32_group_role: tile %dx%d/%d", BM, BN,
                 U);
  }
  const dim3 grid(g.total), block(NT);
  // instantiations: every single kind, the MLP-backward pairs (dgrad + wgrad with / without
  // row sums, two wgrads), else all kinds
  switch (kinds) {
#define K_(M_)                                                                          \
  case M_:                                                                             \
    hipLaunchKernelGGL((gemm_group_kernel<BM, BN, WGM, WGN, M_, U>), grid, block, 0, st, g); \
    break;
    K_(0) K_(1) K_(2) K_(4) K_(8) K_(16) K_(2 | 16) K_(2 | 4) K_(4 | 16)
#undef K_
    default:
      hipLaunchKernelGGL((gemm_group_kernel<BM, BN, WGM, WGN, 31, U>), grid, block, 0, st, g);
  }
  DLRM_LAUNCH_CHECK("dlrm_gemm_f32");
  return DLRM_OK;
}

int launch_generic(const Desc& d, hipStream_t st) {
  GemmParams p{};
  p.M = d.M, p.N = d.N, p.K = d.K, p.alpha = d.alpha;
  p.A = d.A, p.lda = d.lda, p.B = d.B, p.ldb = d.ldb;
  p.C = d.C, p.ldc = d.ldc, p.epi = d.epi, p.bias = d.bias;
  p.aux = d.aux, p.ldaux = d.ldaux, p.ones_col = d.ones_col;
  p.tiles_m = (int)dlrm::ceil_div(p.M, 64);
  p.tiles_n = (int)dlrm::ceil_div(p.N, 64);
  p.splits = 1;
  const bool a_kc = !d.trans_a, b_kc = d.trans_b != 0;
  const dim3 grid(p.tiles_m * p.tiles_n), block(kThreads);
  if (a_kc && b_kc)
    hipLaunchKernelGGL((gemm_generic_kernel<true, true>), grid, block, 0, st, p);
  else if (a_kc)
    hipLaunchKernelGGL((gemm_generic_kernel<true, false>), grid, block, 0, st, p);
  else if (b_kc)
    hipLaunchKernelGGL((gemm_generic_kernel<false, true>), grid, block, 0, st, p);
  else
    hipLaunchKernelGGL((gemm_generic_kernel<false, false>), grid, block, 0, st, p);
  DLRM_LAUNCH_CHECK("dlrm_gemm_f32 (generic)");
  if (d.ones_col >= 0) {
    hipLaunchKernelGGL(gemm_rowsum_kernel, dim3(dlrm::ceil_div(d.M, 64)), dim3(kThreads), 0, st, p,
                       a_kc);
    DLRM_LAUNCH_CHECK("dlrm_gemm_f32 (row sum)");
  }
  return DLRM_OK;
}

int check_desc(const Desc& d) {
  DLRM_ARG(d.mode >= DLRM_GEMM_FULL && d.mode <= DLRM_GEMM_REDUCE, "dlrm_gemm_f32: bad mode");
  if (d.mode != DLRM_GEMM_FULL) {
    DLRM_ARG(d.part, "dlrm_gemm_f32: PARTIAL/REDUCE need a partial buffer");
    DLRM_ARG(d.mode != DLRM_GEMM_REDUCE || (d.splits >= 1 && d.N % 4 == 0 && d.M >= 0 && d.C &&
                                            d.ldc >= d.N),
             "dlrm_gemm_f32: REDUCE needs splits >= 1, N %% 4 == 0 and C");
    if (d.mode == DLRM_GEMM_REDUCE) {
      DLRM_ARG(d.ones_col < 0 || (d.ones_col >= d.N && d.ones_col < d.ldc),
               "dlrm_gemm_f32: ones_col outside [N, ldc)");
      return DLRM_OK;
    }
    DLRM_REQUIRE(pipe_ok(d), DLRM_ERR_UNSUPPORTED,
                 "dlrm_gemm_f32: PARTIAL needs 16-B aligned operands, K %% 4 == 0");
    // the REDUCE job repeats the caller's count: a count the planner would lower (K too
    // short for it, or above kMaxSplit) would leave slabs unwritten
    DLRM_ARG(d.splits <= 0 || make_plan(d.splits, d.K).splits == d.splits,
             "dlrm_gemm_f32: PARTIAL splits=%d is not a normalized count for K=%lld "
             "(use dlrm_gemm_f32_splits)", (int)d.splits, (long long)d.K);
  }
  DLRM_ARG(d.M >= 0 && d.N >= 0 && d.K >= 0, "dlrm_gemm_f32: negative size");
  if (d.M == 0 || (d.N == 0 && d.ones_col < 0)) return DLRM_OK;
  DLRM_ARG(d.C, "dlrm_gemm_f32: null C");
  DLRM_ARG(d.K == 0 || (d.A && d.B), "dlrm_gemm_f32: null A/B");
  DLRM_ARG(d.epi >= DLRM_EPI_STORE && d.epi <= DLRM_EPI_RELU, "dlrm_gemm_f32: bad epilogue");
  DLRM_ARG(!(d.epi == DLRM_EPI_BIAS || d.epi == DLRM_EPI_BIAS_RELU) || d.bias,
           "dlrm_gemm_f32: epilogue needs bias");
  DLRM_ARG(d.epi != DLRM_EPI_DRELU || (d.aux && d.ldaux >= d.N), "dlrm_gemm_f32: DRELU needs aux");
  DLRM_ARG(d.ldc >= d.N && (d.ones_col < 0 || (d.ones_col >= d.N && d.ones_col < d.ldc)),
           "dlrm_gemm_f32: ldc < N or ones_col outside [N, ldc)");
  DLRM_ARG(d.trans_a ? d.lda >= d.M : d.lda >= d.K, "dlrm_gemm_f32: bad lda");
  DLRM_ARG(d.trans_b ? d.ldb >= d.K : d.ldb >= d.N, "dlrm_gemm_f32: bad ldb");
  DLRM_REQUIRE(dlrm::ceil_div(d.M, 64) * dlrm::ceil_div(d.N, 64) < (int64_t)INT32_MAX / kMaxSplit,
               DLRM_ERR_UNSUPPORTED, "dlrm_gemm_f32: too large");
  return DLRM_OK;
}

// Plans n problems: the pipelined group (problems it can take) + generic fallbacks.
size_t ws_for(int n, const Desc* d) {
  Desc q[kMaxGroup];
  int m = 0;
  for (int i = 0; i < n; ++i)
    if (d[i].M > 0 && d[i].N > 0 && d[i].K > 0 && pipe_ok(d[i])) q[m++] = d[i];
  if (m == 0) return 0;
  Tile t;
  Plan pl[kMaxGroup];
  plan_launch(m, q, t, pl);
  const size_t a = group_ws_bytes(m, q, t, pl);
  const size_t b = group_ws_bytes(m, q, Tile{64, 32, 2, 2}, pl);  // as a role launch
  return a > b ? a : b;
}

int run(int n, const Desc* d, void* ws, size_t ws_bytes, hipStream_t st,
        const LaunchRole* role = nullptr, int phase = 0) {
  DLRM_ARG(n >= (role ? 0 : 1) && n <= kMaxGroup, "dlrm_gemm_f32_group: 1..%d problems",
           kMaxGroup);
  Desc q[kMaxGroup];
  int m = 0;
  for (int i = 0; i < n; ++i) {
    const int rc = check_desc(d[i]);
    if (rc != DLRM_OK) return rc;
    if (d[i].M == 0 || (d[i].N == 0 && d[i].ones_col < 0)) continue;
    if (d[i].mode == DLRM_GEMM_REDUCE) {
      q[m++] = d[i];
      continue;
    }
    if (d[i].K == 0 || !pipe_ok(d[i])) {
      const int r2 = launch_generic(d[i], st);
      if (r2 != DLRM_OK) return r2;
      continue;
    }
    q[m++] = d[i];
  }
  if (m == 0 && !role) return DLRM_OK;
  Tile t;
  Plan pl[kMaxGroup];
  plan_launch(m, q, t, pl);
  // a launch carrying an update pass runs 64x32 or 32x64 tiles (gemm_role_kernel; the tile
  // shape does not change any result, ws_for sizes the workspace for 64x32 too)
  if (role && !(t == Tile{64, 32, 2, 2}) && !(t == Tile{32, 64, 2, 2})) {
    if (split_tiles(m, q, Tile{64, 32, 2, 2}, pl) > kTicketCap) {
      // the smaller tile would need more split-K tickets than the workspace head holds:
      // the role's pass runs as its own launch, then the group on its planned tile
      const int rc = launch_group<64, 32>(0, q, pl, ws, ws_bytes, role, phase, st);
      if (rc != DLRM_OK) return rc;
      return run(m, q, ws, ws_bytes, st);
    }
    t = Tile{64, 32, 2, 2};
  }
  const size_t need = group_ws_bytes(m, q, t, pl);
  if (need > 0 && (!ws || ws_bytes < need)) {  // no workspace: in-launch splits off
    // (PARTIAL / REDUCE plans pair with each other across launches: kept)
    for (int i = 0; i < m; ++i)
      if (q[i].mode == DLRM_GEMM_FULL) pl[i] = make_plan(1, q[i].K);
  }
  if (t.bm == 128) return launch_group<128, 64>(m, q, pl, ws, ws_bytes, role, phase, st);
  if (t.bn == 128) return launch_group<64, 128>(m, q, pl, ws, ws_bytes, role, phase, st);
  if (t.bm == 32 && t.bn == 32)
    return launch_group<32, 32>(m, q, pl, ws, ws_bytes, role, phase, st);
  if (t.bm == 32) return launch_group<32, 64>(m, q, pl, ws, ws_bytes, role, phase, st);
  if (t.bn == 32) return launch_group<64, 32>(m, q, pl, ws, ws_bytes, role, phase, st);
  return launch_group<64, 64>(m, q, pl, ws, ws_bytes, role, phase, st);
}

Desc desc_of(const dlrm_gemm_problem& g) {
  Desc d;
  d.trans_a = g.trans_a, d.trans_b = g.trans_b;
  d.M = g.M, d.N = g.N, d.K = g.K, d.alpha = g.alpha;
  d.A = g.A, d.lda = g.lda, d.B = g.B, d.ldb = g.ldb;
  d.C = g.C, d.ldc = g.ldc, d.epi = g.epilogue, d.bias = g.bias;
  d.aux = g.aux, d.ldaux = g.ld_aux, d.ones_col = g.ones_col;
  d.mode = g.mode, d.splits = g.splits, d.part = g.partial;
  return d;
}

}  // namespace

extern "C" size_t dlrm_gemm_f32_workspace_size(int32_t trans_a, int32_t trans_b, int64_t M,
                                               int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  Desc d{};
  d.trans_a = trans_a, d.trans_b = trans_b, d.M = M, d.N = N, d.K = K;
  // aligned, padded placeholders: the size covers any aligned call of this shape
  d.lda = ((trans_a ? M : K) + 3) / 4 * 4, d.ldb = ((trans_b ? K : N) + 3) / 4 * 4;
  d.A = d.B = reinterpret_cast<const float*>(256);
  d.ones_col = -1;
  return ws_for(1, &d);
}

extern "C" int dlrm_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                             float alpha, const float* A, int64_t lda, const float* B,
                             int64_t ldb, float* C, int64_t ldc, int32_t epilogue,
                             const float* bias, const float* aux, int64_t ld_aux,
                             void* workspace, size_t workspace_bytes, dlrm_stream_t stream) {
  Desc d;
  d.trans_a = trans_a, d.trans_b = trans_b, d.M = M, d.N = N, d.K = K, d.alpha = alpha;
  d.A = A, d.lda = lda, d.B = B, d.ldb = ldb, d.C = C, d.ldc = ldc, d.epi = epilogue;
  d.bias = bias, d.aux = aux, d.ldaux = ld_aux, d.ones_col = -1;
  return run(1, &d, workspace, workspace_bytes, dlrm::as_stream(stream));
}

extern "C" size_t dlrm_gemm_f32_group_workspace_size(int32_t n, const dlrm_gemm_problem* probs) {
  if (n < 1 || n > kMaxGroup || !probs) return 0;
  Desc d[kMaxGroup];
  for (int i = 0; i < n; ++i) d[i] = desc_of(probs[i]);
  return ws_for(n, d);
}

extern "C" int dlrm_gemm_f32_group(int32_t n, const dlrm_gemm_problem* probs, void* workspace,
                                   size_t workspace_bytes, dlrm_stream_t stream) {
  DLRM_ARG(probs && n >= 1 && n <= kMaxGroup, "dlrm_gemm_f32_group: 1..%d problems", kMaxGroup);
  Desc d[kMaxGroup];
  for (int i = 0; i < n; ++i) d[i] = desc_of(probs[i]);
  return run(n, d, workspace, workspace_bytes, dlrm::as_stream(stream));
}

extern "C" int dlrm_gemm_f32_group_role(int32_t n, const dlrm_gemm_problem* probs,
                                        void* workspace, size_t workspace_bytes,
                                        const dlrm_launch_role* role, int32_t phase,
                                        dlrm_stream_t stream) {
  const char* name = "dlrm_gemm_f32_group_role";
  const auto* r = reinterpret_cast<const LaunchRole*>(role);
  DLRM_ARG(!r || r->magic == kRoleMagic, "%s: role not filled by dlrm_tbe_backward_defer", name);
  if (!r || r->blocks == 0) {
    if (n == 0) return DLRM_OK;
    return dlrm_gemm_f32_group(n, probs, workspace, workspace_bytes, stream);
  }
  DLRM_ARG(phase == 1 || phase == 2 || phase == 4, "%s: phase must be 1, 2 or 4", name);
  DLRM_ARG(role_kind_of_phase(phase) == r->kind,
           "%s: phase %d does not match the role (1 / 2: dlrm_tbe_backward_defer, 4: "
           "dlrm_head_step_defer)", name, (int)phase);
  DLRM_ARG(n >= 0 && n <= kMaxGroup && (n == 0 || probs), "%s: 0..%d problems", name, kMaxGroup);
  Desc d[kMaxGroup];
  for (int i = 0; i < n; ++i) d[i] = desc_of(probs[i]);
  return run(n, d, workspace, workspace_bytes, dlrm::as_stream(stream), r, phase);
}

extern "C" int32_t dlrm_gemm_f32_splits(const dlrm_gemm_problem* problem) {
  if (!problem) return 0;
  Desc d = desc_of(*problem);
  if (d.mode == DLRM_GEMM_REDUCE) d.mode = DLRM_GEMM_FULL;
  if (d.M <= 0 || d.N <= 0 || d.K <= 0) return 1;
  // PARTIAL with a requested count: that count normalized (what the kernel will run)
  if (d.mode == DLRM_GEMM_PARTIAL && d.splits > 0) return make_plan(d.splits, d.K).splits;
  d.splits = 0;
  Tile t;
  Plan pl;
  plan_one(d, t, pl);
  return pl.splits;
}

extern "C" size_t dlrm_gemm_f32_partial_bytes(int64_t M, int64_t N, int32_t splits) {
  if (M <= 0 || N <= 0 || splits <= 0) return 0;
  return (size_t)splits * (size_t)(M * N + M) * sizeof(float);
}
