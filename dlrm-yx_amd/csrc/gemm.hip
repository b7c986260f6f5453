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

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kThreads = 256;
constexpr int kMaxSplit = 32;
constexpr int kMaxGroup = 4;
constexpr int64_t kTicketCap = 16384;  // int32 tickets in the fixed 64 KiB workspace head
constexpr int kBK = 32;

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
  int pub;           // split-K hand-off: 0 = release/acquire fences, 1 = write-through (sc1)
  int mode;          // DLRM_GEMM_FULL / _PARTIAL (split partials -> part) / _REDUCE
  float* part;       // PARTIAL/REDUCE: [splits][M][N] fp32, then [splits][M] row sums
  // split-bf16 planes (x6d body): [3][rows][ld] bf16 of the stored A / B / C matrices
  const __bf16* Ap;
  int64_t ldap, psa;
  const __bf16* Bp;
  int64_t ldbp, psb;
  __bf16* Cp;        // optional: every epilogue write of C is also split into Cp
  int64_t ldcp, psc;
};

struct GemmGroup {
  GemmParams p[kMaxGroup];
  int n;
  int total;  // blocks in the launch
};

// One operand's (MN x BKT) panel, staged global -> registers -> LDS.
//   KC  : X(mn, k) = X[mn*ld + k]  -> LDS [mn][BKT + 4]   (fragments: ds_read_b128)
//   !KC : X(mn, k) = X[k*ld + mn]  -> LDS [BKT][MN + 4]   (fragments: ds_read_b32)
template <int MN, int BKT, bool KC, bool VEC, int NT>
struct Stage {
  static constexpr int PITCH = KC ? BKT + 4 : MN + 4;
  static constexpr int SIZE = KC ? MN * PITCH : BKT * PITCH;  // floats per LDS buffer
  static constexpr int NV = MN * BKT / 4 / NT;               // float4 per thread
  static_assert(NV >= 1 && MN * BKT % (4 * NT) == 0, "panel / thread mismatch");
  float4 regs[NV];

  __device__ __forceinline__ void coords(int q, int& mn, int& k) const {
    if constexpr (KC) {
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
  // (KC) the columns k >= K of a row and (!KC) the columns mn >= MN of a row, masked here.
  struct Fetch {
    int off[NV];   // byte offset at tile 0 (or -1: masked for every tile)
    int kpos[NV];  // KC: the float4's k within a K-tile
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
    const bool ok = f.off[v] >= 0 && (!KC || kt0 + f.kpos[v] < klim);
    const int off = ok ? f.off[v] + t * tile_step : 0x7ffffff0;
    regs[v] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
  }

  __device__ __forceinline__ void store_one(int v, float* __restrict__ lds, int tid) const {
    int mn, k;
    coords(tid + v * NT, mn, k);
    float* dst = KC ? lds + mn * PITCH + k : lds + k * PITCH + mn;
    *reinterpret_cast<float4*>(dst) = regs[v];
  }

  __device__ __forceinline__ void store(float* __restrict__ lds, int tid) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int mn, k;
      coords(tid + v * NT, mn, k);
      float* dst = KC ? lds + mn * PITCH + k : lds + k * PITCH + mn;
      *reinterpret_cast<float4*>(dst) = regs[v];
    }
  }

  // NS consecutive k-steps (k = kbase .. kbase+NS-1) of the 32-wide sub-tile at `off`
  // for this lane (row/col off + l32).
  template <int NS>
  __device__ __forceinline__ void frag(const float* __restrict__ lds, int off, int l32, int kbase,
                                       float (&f)[NS]) const {
    static_assert(NS % 4 == 0, "fragment length");
    if constexpr (KC) {
      const float* p = lds + (off + l32) * PITCH + kbase;
#pragma unroll
      for (int c = 0; c < NS / 4; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * c);
        f[4 * c + 0] = v.x;
        f[4 * c + 1] = v.y;
        f[4 * c + 2] = v.z;
        f[4 * c + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < NS; ++s) f[s] = lds[(kbase + s) * PITCH + off + l32];
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

// v -> (h, m, l) bf16 bit patterns, v = h + m + l exactly (round to nearest at each level).
__device__ __forceinline__ void split3(float v, unsigned short& h, unsigned short& m,
                                       unsigned short& l) {
  const __bf16 hb = (__bf16)v;
  const float r = v - (float)hb;
  const __bf16 mb = (__bf16)r;
  const __bf16 lb = (__bf16)(r - (float)mb);
  h = __builtin_bit_cast(unsigned short, hb);
  m = __builtin_bit_cast(unsigned short, mb);
  l = __builtin_bit_cast(unsigned short, lb);
}

// v -> the three bf16 planes at Cp (one element).
__device__ __forceinline__ void store_planes(const GemmParams& p, int64_t row, int64_t col,
                                             float v) {
  unsigned short h, m, l;
  split3(v, h, m, l);
  unsigned short* d = reinterpret_cast<unsigned short*>(p.Cp) + row * p.ldcp + col;
  d[0] = h;
  d[p.psc] = m;
  d[2 * p.psc] = l;
}

// N consecutive values (N = 4 or 8) -> the planes at Cp + row*ldcp + col, one 8- / 16-B
// store per plane (col % N == 0; the host guarantees 16-B aligned planes, ldcp % 8 == 0).
template <int N>
__device__ __forceinline__ void store_planes_vec(const GemmParams& p, int64_t row, int64_t col,
                                                 const float* v) {
  unsigned w[3][N / 2];
#pragma unroll
  for (int u = 0; u < N / 2; ++u) {
    unsigned short h0, m0, l0, h1, m1, l1;
    split3(v[2 * u], h0, m0, l0);
    split3(v[2 * u + 1], h1, m1, l1);
    w[0][u] = h0 | ((unsigned)h1 << 16);
    w[1][u] = m0 | ((unsigned)m1 << 16);
    w[2][u] = l0 | ((unsigned)l1 << 16);
  }
  __bf16* d = p.Cp + row * p.ldcp + col;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if constexpr (N == 8)
      *reinterpret_cast<uint4*>(d + q * p.psc) = make_uint4(w[q][0], w[q][1], w[q][2], w[q][3]);
    else
      *reinterpret_cast<uint2*>(d + q * p.psc) = make_uint2(w[q][0], w[q][1]);
  }
}

// C = epilogue(v) where v = alpha * acc (already scaled); returns the value written.
// planes = false: the caller writes the C planes itself (vectorized).
__device__ __forceinline__ float apply_epilogue(const GemmParams& p, int64_t row, int64_t col,
                                                float v, bool planes = true) {
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
  if (planes && p.Cp) store_planes(p, row, col, v);
  return v;
}


// Split-K completion.  Each split workgroup stores its NV accumulators (fragment order,
// thread-major: rec[tid*NV + q]) and its row sums (rec[BM*BN + local row]) into its
// record, then takes a ticket; the last arriver sums every split's record in split order
// and applies the epilogue.  Publication is the agent-scope release/acquire hand-off
// (per-XCD L2s are not coherent): plain stores -> s_waitcnt vmcnt(0) -> barrier ->
// release fence -> vmcnt(0) -> relaxed agent ticket; last arriver: acquire fence ->
// vmcnt(0) -> barrier -> plain loads (unconditional, two splits in flight).  The last
// arriver resets the tile's ticket for the next launch.  Returns true in the workgroup
// that must write the output (always when unsplit); v / rs then hold the full sums.
template <int BM, int BN, int NV, int FM>
__device__ __forceinline__ bool splitk_reduce(const GemmParams& p, int tile, int split,
                                              float (&v)[NV], float (&rs)[FM], int rs_row0,
                                              int rs_stride, bool rs_owner, float* smem) {
  if (p.splits <= 1 || p.pub == 2) return true;  // (pub 2: timing probe only, wrong sums)
  constexpr int REC = BM * BN + BM;
  static_assert(NV % 4 == 0, "record chunks are float4");
  using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
  const int tid = threadIdx.x;
  const bool wt = p.pub == 1;  // write-through records: no fences (MI355X guide, sc1 form)
  float* tile_base = p.ws + (int64_t)tile * p.splits * REC;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)tile_base, (short)0, (int)(p.splits * REC * 4), 0x00020000);
  float* rec = tile_base + (int64_t)split * REC;
  if (wt) {
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
  } else {
#pragma unroll
    for (int q = 0; q < NV; q += 4)
      *reinterpret_cast<float4*>(rec + tid * NV + q) = make_float4(v[q], v[q + 1], v[q + 2], v[q + 3]);
    if (rs_owner) {
#pragma unroll
      for (int i = 0; i < FM; ++i) rec[BM * BN + rs_row0 + i * rs_stride] = rs[i];
    }
  }
  if (p.pub == 3) return split == 0;  // (timing probe only: records stored, no hand-off)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if (!wt) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == p.splits - 1;
    if (last) {
      if (!wt) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    reinterpret_cast<volatile int*>(smem)[0] = last;
  }
  __syncthreads();
  if (!reinterpret_cast<volatile int*>(smem)[0]) return false;
  const int rrow = rs_owner ? rs_row0 : 0;  // every lane loads (valid address), owners use it
  auto load_rec = [&](int s, float4 (&t)[NV / 4], float (&tr)[FM]) {
    const int o = s * REC;
    if (wt) {  // every load of the records is an sc1 load
#pragma unroll
      for (int q = 0; q < NV / 4; ++q)
        t[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rr, (o + tid * NV + 4 * q) * 4, 0, 16));
#pragma unroll
      for (int i = 0; i < FM; ++i)
        tr[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rr, (o + BM * BN + rrow + i * rs_stride) * 4, 0, 16));
    } else {
      const float* r = tile_base + o;
#pragma unroll
      for (int q = 0; q < NV / 4; ++q)
        t[q] = *reinterpret_cast<const float4*>(r + tid * NV + 4 * q);
#pragma unroll
      for (int i = 0; i < FM; ++i) tr[i] = r[BM * BN + rrow + i * rs_stride];
    }
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

// Tile epilogue shared by the fp32 and the split-bf16 bodies: PARTIAL slabs, or the split-K
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
  // C planes: the written tile is staged in LDS (free now) and split in 8-column chunks,
  // one 16-B store per plane (a lane's accumulators are 4 rows of one column)
  constexpr int LDT = BN + 4;
  const bool stage = p.Cp != nullptr;
  if (stage) __syncthreads();  // every wave is done with the main loop's LDS
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = n0 + wn0 + j * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm0 + i * 16 + 4 * kq + r;
        if (row < p.M && col < p.N) {
          const float w = apply_epilogue(p, row, col, p.alpha * v[(i * FN + j) * 4 + r], false);
          if (stage) smem[(wm0 + i * 16 + 4 * kq + r) * LDT + wn0 + j * 16 + l16] = w;
        }
      }
    }
  if (stage) {
    __syncthreads();
    constexpr int NT = WGM * WGN * 64, CPRW = BN / 8;
    for (int c = tid; c < BM * CPRW; c += NT) {
      const int r = c / CPRW, c8 = 8 * (c - r * CPRW);
      const int64_t row = m0 + r, col = n0 + c8;
      if (row >= p.M || col >= p.N) continue;
      const float* src = smem + r * LDT + c8;
      if (col + 8 <= p.N) {
        float w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = src[u];
        store_planes_vec<8>(p, row, col, w);
      } else {
        for (int u = 0; u < 8 && col + u < p.N; ++u) store_planes(p, row, col + u, src[u]);
      }
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
// workgroup is WGM x WGN waves, each owning a (BM/WGM) x (BN/WGN) sub-tile.
template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, bool RS>
__device__ __forceinline__ void pipe_body(const GemmParams& p, int lb, float* smem) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile");
  constexpr int KL = kBK / 4;  // k-steps per K-tile (each lane group owns KL consecutive k)
  using SA = Stage<BM, kBK, A_KC, true, NT>;
  using SB = Stage<BN, kBK, B_KC, true, NT>;
  constexpr int NS = SA::NV + SB::NV;  // staged float4 per thread per K-tile
  static_assert(NS <= KL - 1, "staging must finish before the barrier step");

  const int tile = lb / p.splits;
  const int split = lb - tile * p.splits;
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
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

  const int nk = (int)((kend - kbeg + kBK - 1) / kBK);
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
  const int a_step = A_KC ? kBK * 4 : (int)(kBK * p.lda * 4);
  const int b_step = B_KC ? kBK * 4 : (int)(kBK * p.ldb * 4);
  const int kb32 = (int)kbeg, K32 = (int)p.K;
  auto fetch_one = [&](int c, int t) {  // staged float4 c of K-tile t (unused past nk)
    if (c < SA::NV)
      sa.fetch4(c, fa, ra, a_step, t, kb32 + t * kBK, K32);
    else
      sb.fetch4(c - SA::NV, fb, rb, b_step, t, kb32 + t * kBK, K32);
  };
  auto put_one = [&](int c, float* buf) {
    if (c < SA::NV)
      sa.store_one(c, buf, tid);
    else
      sb.store_one(c - SA::NV, buf + SA::SIZE, tid);
  };
  auto read_frags = [&](const float* buf, float (&a)[FM][KL], float (&b)[FN][KL]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) sa.template frag<KL>(buf, wm0 + i * 16, l16, kq * KL, a[i]);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      sb.template frag<KL>(buf + SA::SIZE, wn0 + j * 16, l16, kq * KL, b[j]);
  };

  float a[FM][KL], b[FN][KL];
  // Prologue: tile 0 -> LDS buffer 0, tile 1 staged in registers, tile 0 fragments read.
  // Every fetch is unconditional: tiles past nk load zeros (their LDS image is never used).
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 0);
#pragma unroll
  for (int c = 0; c < NS; ++c) put_one(c, smem);
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 1);
  __syncthreads();
  read_frags(smem, a, b);

  // One K-tile: MFMAs on (ca, cb) with the staging of tile t+1 / fetch of t+2 interleaved,
  // barrier, then tile t+1's fragments into (na, nb) under the last k-step.  The loop is
  // unrolled by two so the fragment sets ping-pong without register copies.
  auto iteration = [&](int kt, float (&ca)[FM][KL], float (&cb)[FN][KL], float (&na)[FM][KL],
                       float (&nb)[FN][KL]) {
    float* nbuf = smem + ((kt + 1) & 1) * (SA::SIZE + SB::SIZE);
#pragma unroll
    for (int s = 0; s < KL - 1; ++s) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[i][s], cb[j][s], acc[i][j], 0, 0, 0);
      if constexpr (RS) {
#pragma unroll
        for (int i = 0; i < FM; ++i) rs[i] = add_f32(rs[i], ca[i][s]);
      }
      if (s < NS) {
        put_one(s, nbuf);      // tile t+1 (staged last iteration) -> LDS
        fetch_one(s, kt + 2);  // refill the register with tile t+2
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the interleave: no hoisting across steps
    }
    __syncthreads();  // tile t+1 is complete in LDS
    read_frags(nbuf, na, nb);
    __builtin_amdgcn_sched_barrier(0);  // issue the reads before the last step's MFMAs
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[i][KL - 1], cb[j][KL - 1], acc[i][j],
                                                         0, 0, 0);
    if constexpr (RS) {
#pragma unroll
      for (int i = 0; i < FM; ++i) rs[i] = add_f32(rs[i], ca[i][KL - 1]);
    }
  };
  float a1[FM][KL], b1[FN][KL];
  for (int kt = 0; kt < nk; kt += 2) {
    iteration(kt, a, b, a1, b1);
    if (kt + 1 >= nk) break;
    iteration(kt + 1, a1, b1, a, b);
  }

  // Row sums: lanes l16, l16+16, l16+32, l16+48 hold the four k-quarters of row l16
  // (fixed pairing order: deterministic).
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
  }
  finish_tile<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0, smem);
}

// ------------------------------------------------------------- LDS-DMA f32 body --
// The second fp32 body (r03), picked per shape by the plan: operand panels go global -> LDS by LDS-DMA
// (buffer_load_dwordx4 ... lds, 1 KiB per wave instruction) through a kStages-deep ring,
// so kStages - 1 K-tiles are in flight with no staging registers and no ds_write; the
// fragments of K-tile t+1 are read under the second half of tile t's MFMAs (one barrier
// per K-tile).  A/B against the register-staged pipe_body (DLRM_GEMM_BODY=reg):
// profiles/r03_gemm_dma_probe.txt (C3 shapes 5-20 % faster).
// LDS images (1 KiB blocks, bank maps checked offline: every ds_read group touches 64
// distinct banks):
//   KC  : 8 rows x 32 k per block; row r's 16-B chunk c in slot 8 (r % 8) + (c ^ s(r)),
//         s(r) = (r ^ (r >> 3)) & 7  (fragment reads: ds_read_b128);
//   !KC : 256/MN k-rows x MN per block; chunk c of row k in slot (k % rpb)(MN/4) + (c ^ g(k)),
//         g(k) = 4 ((k >> 3) & 1) mod MN/4  (fragment reads: ds_read_b32).
constexpr int kStages = 4;
typedef __attribute__((address_space(3))) const float lds_cfloat;

template <int MN, bool KC>
struct DImg {
  static constexpr int FLOATS = MN * kBK;           // one stage
  static constexpr int BLOCKS = FLOATS * 4 / 1024;  // KiB blocks (one DMA instruction each)
  static constexpr int CPR = MN / 4;                // !KC: 16-B chunks per k-row
  static constexpr int RPB = KC ? 8 : 256 / MN;     // rows per block
  __device__ __forceinline__ static int swz(int r) { return (r ^ (r >> 3)) & 7; }
  __device__ __forceinline__ static int g(int k) { return (4 * ((k >> 3) & 1)) % CPR; }
  // (mn, k) of the 16-B chunk lane l of block b loads
  __device__ __forceinline__ static void lane_src(int b, int l, int& mn, int& k) {
    if constexpr (KC) {
      mn = b * 8 + (l >> 3);
      k = 4 * ((l & 7) ^ swz(mn));
    } else {
      k = b * RPB + l / CPR;
      mn = 4 * ((l % CPR) ^ g(k));
    }
  }
  __device__ __forceinline__ static int at(int mn, int k) {  // float offset in the stage
    if constexpr (KC)
      return (mn >> 3) * 256 + ((mn & 7) * 8 + ((k >> 2) ^ swz(mn))) * 4 + (k & 3);
    else
      return (k / RPB) * 256 + ((k % RPB) * CPR + ((mn >> 2) ^ g(k))) * 4 + (mn & 3);
  }
};

// One LDS-DMA wave instruction (64 lanes x 16 B -> LDS [lds, +1 KiB)) in inline asm: the
// compiler's waitcnt pass does not see it as an LDS store, so it does not drain every
// in-flight DMA (vmcnt(0)) before the next ds_read of ANOTHER ring stage; wait_vm<N>
// orders instead.  (M0 is reserved by the compiler, which keeps no value in it here.)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const float* lds, int voff) {
  const unsigned a = (unsigned)(uintptr_t)(lds_cfloat*)lds;
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(a),
               "v"(voff), "s"(r)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN>
constexpr int dma_smem_floats() {
  return kStages * (BM + BN) * kBK;
}

template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, bool RS>
__device__ __forceinline__ void pipe_body_dma(const GemmParams& p, int lb, float* smem) {
  constexpr int S = kStages;
  constexpr int WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
  constexpr int NW = WGM * WGN;
  constexpr int KL = kBK / 4;
  using IA = DImg<BM, A_KC>;
  using IB = DImg<BN, B_KC>;
  constexpr int STAGE = IA::FLOATS + IB::FLOATS;
  static_assert(IA::BLOCKS % NW == 0 && IB::BLOCKS % NW == 0, "DMA blocks per wave");
  constexpr int NIA = IA::BLOCKS / NW, NIB = IB::BLOCKS / NW;  // DMA instrs per wave / tile
  constexpr int NI = NIA + NIB;

  const int tile = lb / p.splits;
  const int split = lb - tile * p.splits;
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, l16 = lane & 15;
  const int wm0 = (wave / WGN) * WM, wn0 = (wave % WGN) * WN;
  const int nk = (int)((kend - kbeg + kBK - 1) / kBK);

  const int64_t a_ext = A_KC ? (p.M - 1) * p.lda + p.K : (p.K - 1) * p.lda + p.M;
  const int64_t b_ext = B_KC ? (p.N - 1) * p.ldb + p.K : (p.K - 1) * p.ldb + p.N;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)(a_ext * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)(b_ext * 4), 0x00020000);
  // per DMA instruction of this wave: byte offset at the split's first K-tile (-1: the
  // row / column is outside the operand), the chunk's k within a tile
  int aoff[NIA], akp[NIA], boff[NIB], bkp[NIB];
#pragma unroll
  for (int i = 0; i < NIA; ++i) {
    int mn, k;
    IA::lane_src(wave * NIA + i, lane, mn, k);
    const int64_t gmn = m0 + mn, gk = kbeg + k;
    aoff[i] = gmn < p.M ? (int)(4 * (A_KC ? gmn * p.lda + gk : gk * p.lda + gmn)) : -1;
    akp[i] = k;
  }
#pragma unroll
  for (int i = 0; i < NIB; ++i) {
    int mn, k;
    IB::lane_src(wave * NIB + i, lane, mn, k);
    const int64_t gmn = n0 + mn, gk = kbeg + k;
    boff[i] = gmn < p.N ? (int)(4 * (B_KC ? gmn * p.ldb + gk : gk * p.ldb + gmn)) : -1;
    bkp[i] = k;
  }
  const int a_step = A_KC ? 4 * kBK : (int)(4 * kBK * p.lda);
  const int b_step = B_KC ? 4 * kBK : (int)(4 * kBK * p.ldb);
  const int krem = (int)(kend - kbeg);  // k range of this split
  // DMA of K-tile t into stage t % S; tiles past the split (t >= nk) and chunks past K load
  // zeros (out-of-descriptor offset), so every wave issues the same instruction count
  auto issue = [&](int t) {
    float* st = smem + (t % S) * STAGE;
#pragma unroll
    for (int i = 0; i < NIA; ++i) {
      const bool ok = aoff[i] >= 0 && t * kBK + akp[i] < krem;
      dma16(ra, st + (wave * NIA + i) * 256, ok ? aoff[i] + t * a_step : 0x7ffffff0);
    }
#pragma unroll
    for (int i = 0; i < NIB; ++i) {
      const bool ok = boff[i] >= 0 && t * kBK + bkp[i] < krem;
      dma16(rb, st + IA::FLOATS + (wave * NIB + i) * 256, ok ? boff[i] + t * b_step : 0x7ffffff0);
    }
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rs[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) rs[i] = 0.f;
  auto read = [&](int t, float (&a)[FM][KL], float (&b)[FN][KL]) {
    const float* st = smem + (t % S) * STAGE;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int mn = wm0 + i * 16 + l16;
#pragma unroll
      for (int s = 0; s < KL; s += (A_KC ? 4 : 1)) {
        if constexpr (A_KC) {
          const float4 v = *reinterpret_cast<const float4*>(st + IA::at(mn, kq * KL + s));
          a[i][s] = v.x, a[i][s + 1] = v.y, a[i][s + 2] = v.z, a[i][s + 3] = v.w;
        } else {
          a[i][s] = st[IA::at(mn, kq * KL + s)];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int mn = wn0 + j * 16 + l16;
#pragma unroll
      for (int s = 0; s < KL; s += (B_KC ? 4 : 1)) {
        if constexpr (B_KC) {
          const float4 v =
              *reinterpret_cast<const float4*>(st + IA::FLOATS + IB::at(mn, kq * KL + s));
          b[j][s] = v.x, b[j][s + 1] = v.y, b[j][s + 2] = v.z, b[j][s + 3] = v.w;
        } else {
          b[j][s] = st[IA::FLOATS + IB::at(mn, kq * KL + s)];
        }
      }
    }
  };
  auto mfma = [&](const float (&a)[FM][KL], const float (&b)[FN][KL], int s0, int s1) {
#pragma unroll
    for (int s = s0; s < s1; ++s) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
      if constexpr (RS) {
#pragma unroll
        for (int i = 0; i < FM; ++i) rs[i] = add_f32(rs[i], a[i][s]);
      }
    }
  };
  float ca[FM][KL], cb[FN][KL], na[FM][KL], nb[FN][KL];
#pragma unroll
  for (int t = 0; t < S - 1; ++t) issue(t);
  wait_vm<(S - 2) * NI>();       // tile 0 landed (this wave)
  __builtin_amdgcn_s_barrier();  // (every wave; a bare barrier: __syncthreads' fence would
  asm volatile("" ::: "memory");  //  drain every DMA in flight)
  read(0, ca, cb);
  auto step = [&](int t, float (&a)[FM][KL], float (&b)[FN][KL], float (&a2)[FM][KL],
                  float (&b2)[FN][KL]) {
    mfma(a, b, 0, KL / 2);
    wait_vm<(S - 3) * NI>();       // tile t+1 landed (this wave)
    __builtin_amdgcn_s_barrier();  // every wave's has; every wave has read tile t-1's stage
    asm volatile("" ::: "memory");
    issue(t + S - 1);  // into tile t-1's stage
    read(t + 1, a2, b2);
    mfma(a, b, KL / 2, KL);
  };
  for (int t = 0; t < nk; t += 2) {
    step(t, ca, cb, na, nb);
    if (t + 1 >= nk) break;
    step(t + 1, na, nb, ca, cb);
  }
  wait_vm<0>();  // the trailing DMAs (tiles >= nk) land before smem is reused or released
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
  }
  finish_tile<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0, smem);
}

// ---------------------------------------------------------------- split-bf16 body --
// fp32 GEMM on the bf16 matrix core (v_mfma_f32_16x16x32_bf16, 16x the f32 MFMA rate).
// Every fp32 operand x is split exactly into three bf16 terms, x = h + m + l (round to
// nearest at each level: |m| <= 2^-8 |x|, |l| <= 2^-16 |x|, and l is exact because the
// residual after two 8-bit roundings has at most 8 significant bits).  A product is then
//   a*b = ah*bh + (ah*bm + am*bh) + (ah*bl + al*bh + am*bm) + O(2^-24 |a*b|),
// six bf16 products whose dropped terms (am*bl, al*bm, al*bl) are below one fp32 ulp of
// a*b.  The products are exact in the MFMA and accumulate in fp32, 6 roundings per 32 k
// (the f32 MFMA rounds once per k), so the result is as accurate as the exact-f32 path
// (tests/test_gpu_kernels.py::test_gemm_x6_accuracy bounds both against fp64).
//
// Staging is the fp32 body's (raw buffer loads of whole float4s); the split happens once
// per element when a thread writes its staged float4 to LDS, as three bf16 planes:
//   k-contiguous operand  -> [mn][32 + 8]  per plane, fragments by ds_read_b128;
//   mn-contiguous operand -> [k/8][8][MN + 16] (+32 dwords between k-octets) per plane,
//   fragments by two ds_read_b64_tr_b16 (hardware transpose; the pitch and the octet gap
//   put the eight rows a 32-lane half reads on eight distinct 8-bank windows).
// One K-tile (BK = 32) is one 16x16x32 k-step: lane l holds k = 8(l>>4) .. +7 of row /
// column l&15 for both operands, the map of the fp32 body's fragments.
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using s16x4 = __attribute__((ext_vector_type(4))) short;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ unsigned pk_bf16(float x0, float x1) {
  using bf16x2 = __attribute__((ext_vector_type(2))) __bf16;
  return __builtin_bit_cast(unsigned, bf16x2{(__bf16)x0, (__bf16)x1});  // v_cvt_pk_bf16_f32
}
__device__ __forceinline__ float lo_f(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float hi_f(unsigned u) {
  return __builtin_bit_cast(float, u & 0xffff0000u);
}
// The conversion is opaque inline asm so the compiler keeps lo_f(h) as one shift (left to
// itself it re-converts x0 alone); gemm.hip is built with -fno-slp-vectorize so the two
// subtractions stay v_sub_f32 (a v_pk_add_f32 beside MFMAs costs ~26 cycles per gap).
__device__ __forceinline__ unsigned cvt_pk_bf16(float a, float b) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// x0, x1 -> packed (h, m, l) bf16 pairs, x = h + m + l exactly.
__device__ __forceinline__ void split2(float x0, float x1, unsigned& h, unsigned& m,
                                       unsigned& l) {
  h = cvt_pk_bf16(x0, x1);
  const float r0 = x0 - lo_f(h), r1 = x1 - hi_f(h);
  m = cvt_pk_bf16(r0, r1);
  const float s0 = r0 - lo_f(m), s1 = r1 - hi_f(m);
  l = cvt_pk_bf16(s0, s1);
}

// bf16 three-plane image of one operand's (MN x 32) panel (one LDS buffer).
template <int MN, bool KC>
struct Img6 {
  static constexpr int BK = kBK;
  static constexpr int PITCH = KC ? BK + 8 : MN + 16;    // bf16 per row
  static constexpr int OCT = 8 * PITCH + 64;             // !KC: bf16 per k-octet (+32 dwords)
  static constexpr int PLANE = KC ? MN * PITCH : (BK / 8) * OCT;
  static constexpr int SIZE = 3 * PLANE;                 // bf16 per buffer
  static_assert(KC || (PITCH / 16) % 2 == 1, "tr-read pitch must be an odd multiple of 8 dwords");

  // staged float4 (4 consecutive k at mn if KC, 4 consecutive mn at k otherwise) -> planes
  __device__ __forceinline__ static void store(__bf16* buf, int mn, int k, float4 f) {
    unsigned h0, m0, l0, h1, m1, l1;
    split2(f.x, f.y, h0, m0, l0);
    split2(f.z, f.w, h1, m1, l1);
    const int e = KC ? mn * PITCH + k : (k >> 3) * OCT + (k & 7) * PITCH + mn;
    *reinterpret_cast<uint2*>(buf + e) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(buf + PLANE + e) = make_uint2(m0, m1);
    *reinterpret_cast<uint2*>(buf + 2 * PLANE + e) = make_uint2(l0, l1);
  }

  // Fragment of the 16-wide sub-tile at mn0 for this lane: plane q, k = 8 kq .. 8 kq + 7.
  __device__ __forceinline__ static bf16x8 frag(const __bf16* buf, int q, int mn0, int l16,
                                                int kq) {
    const __bf16* pl = buf + q * PLANE;
    if constexpr (KC) {
      return __builtin_bit_cast(
          bf16x8, *reinterpret_cast<const uint4*>(pl + (mn0 + l16) * PITCH + kq * 8));
    } else {
      // ds_read_b64_tr_b16: lane 4r+c of the 16-lane group addresses row r, columns 4c..4c+3
      // of a 4 x 16 block; lane i receives column i, row r in element r.
      const int r = l16 >> 2, c = l16 & 3;
      const __bf16* b0 = pl + kq * OCT + r * PITCH + mn0 + 4 * c;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0 + 4 * PITCH));
      using s16x8 = __attribute__((ext_vector_type(8))) short;
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

template <int BM, int BN>
constexpr int x6_smem_bytes() {
  constexpr int a = Img6<BM, true>::SIZE > Img6<BM, false>::SIZE ? Img6<BM, true>::SIZE
                                                                  : Img6<BM, false>::SIZE;
  constexpr int b = Img6<BN, true>::SIZE > Img6<BN, false>::SIZE ? Img6<BN, true>::SIZE
                                                                  : Img6<BN, false>::SIZE;
  return 2 * (a + b) * 2;  // double-buffered, 2 B per bf16
}

template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, bool RS>
__device__ __forceinline__ void pipe_body6(const GemmParams& p, int lb, float* smem) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile");
  using SA = Stage<BM, kBK, A_KC, true, NT>;
  using SB = Stage<BN, kBK, B_KC, true, NT>;
  using IA = Img6<BM, A_KC>;
  using IB = Img6<BN, B_KC>;
  constexpr int BUF = IA::SIZE + IB::SIZE;  // bf16 per LDS buffer
  constexpr int NS = SA::NV + SB::NV;       // staged float4 per thread per K-tile
  constexpr int NP = 6;                     // bf16 products per K-tile
  static_assert(NS <= NP - 1, "staging must finish before the barrier step");
  static_assert(!RS || !A_KC, "row sums are taken on the mn-contiguous A (wgrad)");

  const int tile = lb / p.splits;
  const int split = lb - tile * p.splits;
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
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
  __bf16* lds = reinterpret_cast<__bf16*>(smem);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 rsq[SA::NV];  // RS: this thread's staged A float4s summed over its k rows
#pragma unroll
  for (int v = 0; v < SA::NV; ++v) rsq[v] = make_float4(0.f, 0.f, 0.f, 0.f);

  const int nk = (int)((kend - kbeg + kBK - 1) / kBK);
  SA sa;
  SB sb;
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
  const int a_step = A_KC ? kBK * 4 : (int)(kBK * p.lda * 4);
  const int b_step = B_KC ? kBK * 4 : (int)(kBK * p.ldb * 4);
  const int kb32 = (int)kbeg, K32 = (int)p.K;
  auto fetch_one = [&](int c, int t) {
    if (c < SA::NV)
      sa.fetch4(c, fa, ra, a_step, t, kb32 + t * kBK, K32);
    else
      sb.fetch4(c - SA::NV, fb, rb, b_step, t, kb32 + t * kBK, K32);
  };
  auto put_one = [&](int c, __bf16* buf, bool live) {  // live: the tile is < nk
    int mn, k;
    if (c < SA::NV) {
      sa.coords(tid + c * NT, mn, k);
      IA::store(buf, mn, k, sa.regs[c]);
      if (RS && live) {
        rsq[c].x = add_f32(rsq[c].x, sa.regs[c].x);
        rsq[c].y = add_f32(rsq[c].y, sa.regs[c].y);
        rsq[c].z = add_f32(rsq[c].z, sa.regs[c].z);
        rsq[c].w = add_f32(rsq[c].w, sa.regs[c].w);
      }
    } else {
      sb.coords(tid + (c - SA::NV) * NT, mn, k);
      IB::store(buf + IA::SIZE, mn, k, sb.regs[c - SA::NV]);
    }
  };
  struct Frag {
    bf16x8 q[3];
  };
  auto read_frags = [&](const __bf16* buf, Frag (&a)[FM], Frag (&b)[FN]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i].q[q] = IA::frag(buf, q, wm0 + i * 16, l16, kq);
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j].q[q] = IB::frag(buf + IA::SIZE, q, wn0 + j * 16, l16, kq);
    }
  };
  // product s of the six: (a plane, b plane), small terms first, h*h last
  auto products = [&](int s, const Frag (&ca)[FM], const Frag (&cb)[FN]) {
    constexpr int PA[NP] = {0, 2, 1, 0, 1, 0};
    constexpr int PB[NP] = {2, 0, 1, 1, 0, 0};
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[i].q[PA[s]], cb[j].q[PB[s]],
                                                            acc[i][j], 0, 0, 0);
  };

  Frag a[FM], b[FN];
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 0);
#pragma unroll
  for (int c = 0; c < NS; ++c) put_one(c, lds, true);
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 1);
  __syncthreads();
  read_frags(lds, a, b);

  auto iteration = [&](int kt, const Frag (&ca)[FM], const Frag (&cb)[FN], Frag (&na)[FM],
                       Frag (&nb)[FN]) {
    __bf16* nbuf = lds + ((kt + 1) & 1) * BUF;
#pragma unroll
    for (int s = 0; s < NP - 1; ++s) {
      products(s, ca, cb);
      if (s < NS) {
        put_one(s, nbuf, kt + 1 < nk);
        fetch_one(s, kt + 2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    read_frags(nbuf, na, nb);
    __builtin_amdgcn_sched_barrier(0);
    products(NP - 1, ca, cb);
  };
  Frag a1[FM], b1[FN];
  for (int kt = 0; kt < nk; kt += 2) {
    iteration(kt, a, b, a1, b1);
    if (kt + 1 >= nk) break;
    iteration(kt + 1, a1, b1, a, b);
  }

  float rs[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) rs[i] = 0.f;
  if constexpr (RS) {
    // Row sums of op(A) = A[k][m]: thread tid staged the mn quad 4*(tid % (BM/4)) at k rows
    // tid / (BM/4) + v*R; sum its float4s (v order), then the R partials per row in order.
    constexpr int Q = BM / 4, R = NT / Q;
    static_assert(NT % Q == 0, "row-sum map");
    float4 t = rsq[0];
#pragma unroll
    for (int v = 1; v < SA::NV; ++v) {
      t.x = add_f32(t.x, rsq[v].x);
      t.y = add_f32(t.y, rsq[v].y);
      t.z = add_f32(t.z, rsq[v].z);
      t.w = add_f32(t.w, rsq[v].w);
    }
    __syncthreads();  // every wave is done with the LDS images
    float* part = smem;  // [R][BM]
    *reinterpret_cast<float4*>(part + (tid / Q) * BM + 4 * (tid % Q)) = t;
    __syncthreads();
    float* sums = smem + R * BM;  // [BM]
    if (tid < BM) {
      float s = part[tid];
      for (int r = 1; r < R; ++r) s += part[r * BM + tid];
      sums[tid] = s;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i) rs[i] = sums[wm0 + i * 16 + l16];
    __syncthreads();  // the split-K hand-off reuses smem[0]
  }
  finish_tile<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0, smem);
}

// ------------------------------------------------- split-bf16 body, 128x128 tiles --
// The x6 math of pipe_body6 on v_mfma_f32_32x32x16_bf16, 128x128 workgroup tiles on 2x2
// waves (64x64 per wave, one wave per SIMD).  Why this shape: the split costs ~22 VALU
// cycles per 64 staged elements and an MFMA leaves the SIMD's vector issue free for 24 of
// its 32 cycles (32x32x16; 8 of 16 on 16x16x32), so the split fits beside the MFMAs only
// when a tile does enough MFMA work per staged element: (BM + BN) / (BM * BN) small.  At
// 64x64 / 16x16x32 (pipe_body6) the split needs ~1.8x the free issue cycles (VALU-bound);
// at 128x128 / 32x32x16 it needs ~0.6x.  Fewer, larger tiles are made up by split-K (the
// plan's split count, in-launch or PARTIAL).
// Measured (profiles/r03_x6l_ab.txt, r03_x6l_pmc.txt): accurate (max error below the f32
// body's) but no faster than the exact-f32 body on the C3 shapes - the split's VALU issue
// (~250 instructions per K-tile and wave) exceeds the 24 free issue cycles per MFMA, and
// 128x128 tiles fill only half the CUs at M = 2048 unless K is split.  Kept as an A/B body
// (DLRM_GEMM_MATH=x6l, plan entries with x6 = 2); the default plan does not use it.
// Per K-tile (32 k) a 64x64 wave runs 2 k16-steps x 6 products x 2x2 tiles = 48 MFMAs (1536
// cycles); the step-1 fragments are read under step 0, the next tile's step-0 fragments
// after the barrier under the last product of step 1; staging of tile t+1 (split to three
// planes on the way into LDS) and the fetch of tile t+2 ride between the MFMA groups.
// LDS images: Img6 with the !KC pitch MN + 32 (row stride = 16 dwords mod 64): the two
// 16-lane groups of a half-wave read columns +0 / +16 of the same four k rows with
// ds_read_b64_tr_b16 on disjoint banks; KC rows of 40 bf16 (20 dwords) keep a 16-lane
// ds_read_b128 group on 64 distinct banks.
template <int MN, bool KC>
struct Img6L {
  static constexpr int BK = kBK;
  static constexpr int PITCH = KC ? BK + 8 : MN + 32;  // bf16 per row
  static constexpr int OCT = 8 * PITCH;                // !KC: bf16 per k-octet
  static constexpr int PLANE = KC ? MN * PITCH : (BK / 8) * OCT;
  static constexpr int SIZE = 3 * PLANE;  // bf16 per buffer

  __device__ __forceinline__ static void store(__bf16* buf, int mn, int k, float4 f) {
    unsigned h0, m0, l0, h1, m1, l1;
    split2(f.x, f.y, h0, m0, l0);
    split2(f.z, f.w, h1, m1, l1);
    const int e = KC ? mn * PITCH + k : (k >> 3) * OCT + (k & 7) * PITCH + mn;
    *reinterpret_cast<uint2*>(buf + e) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(buf + PLANE + e) = make_uint2(m0, m1);
    *reinterpret_cast<uint2*>(buf + 2 * PLANE + e) = make_uint2(l0, l1);
  }

  // 32x32x16 operand fragment of the 32-wide sub-tile at mn0, k16-step `step` of the
  // K-tile: lane l holds mn0 + (l & 31), k = 16 step + 8 (l >> 5) .. +7 of plane q.
  __device__ __forceinline__ static bf16x8 frag(const __bf16* buf, int q, int mn0, int lane,
                                                int step) {
    const __bf16* pl = buf + q * PLANE;
    if constexpr (KC) {
      return __builtin_bit_cast(
          bf16x8, *reinterpret_cast<const uint4*>(pl + (mn0 + (lane & 31)) * PITCH + 16 * step +
                                                  8 * (lane >> 5)));
    } else {
      // 16-lane group g: columns mn0 + 16 (g & 1) .. +15, k-octet 2 step + (g >> 1); lane
      // 4r+c of the group addresses row r, columns 4c..4c+3 (ds_read_b64_tr_b16)
      const int l16 = lane & 15, r = l16 >> 2, c = l16 & 3;
      const __bf16* b0 = pl + (2 * step + (lane >> 5)) * OCT + r * PITCH + mn0 +
                         16 * ((lane >> 4) & 1) + 4 * c;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b0 + 4 * PITCH));
      using s16x8 = __attribute__((ext_vector_type(8))) short;
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

template <int BM, int BN>
constexpr int x6l_smem_bytes() {
  constexpr int a = Img6L<BM, true>::SIZE > Img6L<BM, false>::SIZE ? Img6L<BM, true>::SIZE
                                                                    : Img6L<BM, false>::SIZE;
  constexpr int b = Img6L<BN, true>::SIZE > Img6L<BN, false>::SIZE ? Img6L<BN, true>::SIZE
                                                                    : Img6L<BN, false>::SIZE;
  return 2 * (a + b) * 2;  // double-buffered, 2 B per bf16
}

// finish_tile for 32x32 accumulators (register r of lane l: row 8 (r >> 2) + 4 (l >> 5) +
// (r & 3), column l & 31); rs[i] is the row sum of row wm0 + 32 i + (l & 31).
template <int BM, int BN, int WGM, int WGN, bool RS, int FM, int FN>
__device__ __forceinline__ void finish_tile32(const GemmParams& p, const f32x16 (&acc)[FM][FN],
                                              float (&rs)[FM], int tile, int split, int tn,
                                              int64_t m0, int64_t n0, float* smem) {
  constexpr int WM = BM / WGM, WN = BN / WGN;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int hi = lane >> 5;
  const int l32 = lane & 31;
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;
  const bool rs_owner = RS && tn == 0 && (wave % WGN) == 0 && hi == 0;
  constexpr int NV = FM * FN * 16;
  float v[NV];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) v[(i * FN + j) * 16 + r] = acc[i][j][r];
  auto row_of = [&](int i, int r) -> int64_t {
    return m0 + wm0 + i * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
  };
  if (p.mode == DLRM_GEMM_PARTIAL) {
    float* slab = p.part + (int64_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t col = n0 + wn0 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = row_of(i, r);
          if (row < p.M && col < p.N) slab[row * p.N + col] = v[(i * FN + j) * 16 + r];
        }
      }
    if (rs_owner) {
      float* rslab = p.part + (int64_t)p.splits * p.M * p.N + (int64_t)split * p.M;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int64_t row = m0 + wm0 + i * 32 + l32;
        if (row < p.M) rslab[row] = rs[i];
      }
    }
    return;
  }
  if (!splitk_reduce<BM, BN, NV, FM>(p, tile, split, v, rs, wm0 + l32, 32, rs_owner, smem))
    return;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = n0 + wn0 + j * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = row_of(i, r);
        if (row < p.M && col < p.N)
          apply_epilogue(p, row, col, p.alpha * v[(i * FN + j) * 16 + r]);
      }
    }
  if (rs_owner) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int64_t row = m0 + wm0 + i * 32 + l32;
      if (row < p.M) apply_epilogue(p, row, p.ones_col, p.alpha * rs[i]);
    }
  }
}

template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, bool RS>
__device__ __forceinline__ void pipe_body6L(const GemmParams& p, int lb, float* smem) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int FM = WM / 32, FN = WN / 32;
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile");
  using SA = Stage<BM, kBK, A_KC, true, NT>;
  using SB = Stage<BN, kBK, B_KC, true, NT>;
  using IA = Img6L<BM, A_KC>;
  using IB = Img6L<BN, B_KC>;
  constexpr int BUF = IA::SIZE + IB::SIZE;  // bf16 per LDS buffer
  constexpr int NS = SA::NV + SB::NV;       // staged float4 per thread per K-tile
  constexpr int NP = 6;                     // bf16 products per k16-step
  static_assert(NS <= 2 * NP - 1, "staging must finish before the barrier");
  static_assert(!RS || !A_KC, "row sums are taken on the mn-contiguous A (wgrad)");

  const int tile = lb / p.splits;
  const int split = lb - tile * p.splits;
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wm0 = (wave / WGN) * WM;
  const int wn0 = (wave % WGN) * WN;
  __bf16* lds = reinterpret_cast<__bf16*>(smem);

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float4 rsq[SA::NV];  // RS: this thread's staged A float4s summed over its k rows
#pragma unroll
  for (int v = 0; v < SA::NV; ++v) rsq[v] = make_float4(0.f, 0.f, 0.f, 0.f);

  const int nk = (int)((kend - kbeg + kBK - 1) / kBK);
  SA sa;
  SB sb;
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
  const int a_step = A_KC ? kBK * 4 : (int)(kBK * p.lda * 4);
  const int b_step = B_KC ? kBK * 4 : (int)(kBK * p.ldb * 4);
  const int kb32 = (int)kbeg, K32 = (int)p.K;
  auto fetch_one = [&](int c, int t) {
    if (c < SA::NV)
      sa.fetch4(c, fa, ra, a_step, t, kb32 + t * kBK, K32);
    else
      sb.fetch4(c - SA::NV, fb, rb, b_step, t, kb32 + t * kBK, K32);
  };
  auto put_one = [&](int c, __bf16* buf, bool live) {  // live: the tile is < nk
    int mn, k;
    if (c < SA::NV) {
      sa.coords(tid + c * NT, mn, k);
      IA::store(buf, mn, k, sa.regs[c]);
      if (RS && live) {
        rsq[c].x = add_f32(rsq[c].x, sa.regs[c].x);
        rsq[c].y = add_f32(rsq[c].y, sa.regs[c].y);
        rsq[c].z = add_f32(rsq[c].z, sa.regs[c].z);
        rsq[c].w = add_f32(rsq[c].w, sa.regs[c].w);
      }
    } else {
      sb.coords(tid + (c - SA::NV) * NT, mn, k);
      IB::store(buf + IA::SIZE, mn, k, sb.regs[c - SA::NV]);
    }
  };
  struct Frag {
    bf16x8 q[3];
  };
  auto read_frags = [&](const __bf16* buf, int step, Frag (&a)[FM], Frag (&b)[FN]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i].q[q] = IA::frag(buf, q, wm0 + i * 32, lane, step);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j].q[q] = IB::frag(buf + IA::SIZE, q, wn0 + j * 32, lane, step);
    }
  };
  auto products = [&](int s, const Frag (&ca)[FM], const Frag (&cb)[FN]) {
    constexpr int PA[NP] = {0, 2, 1, 0, 1, 0};
    constexpr int PB[NP] = {2, 0, 1, 1, 0, 0};
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ca[i].q[PA[s]], cb[j].q[PB[s]],
                                                            acc[i][j], 0, 0, 0);
  };

  Frag a0[FM], b0[FN], a1[FM], b1[FN];
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 0);
#pragma unroll
  for (int c = 0; c < NS; ++c) put_one(c, lds, true);
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 1);
  __syncthreads();
  read_frags(lds, 0, a0, b0);

  for (int kt = 0; kt < nk; ++kt) {
    const __bf16* cbuf = lds + (kt & 1) * BUF;
    __bf16* nbuf = lds + ((kt + 1) & 1) * BUF;
    const bool live = kt + 1 < nk;
    read_frags(cbuf, 1, a1, b1);  // step 1 of this tile, consumed after step 0
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      products(s, a0, b0);
      if (s < NS) {
        put_one(s, nbuf, live);  // tile t+1 (staged last iteration) -> LDS planes
        fetch_one(s, kt + 2);    // refill with tile t+2
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int s = 0; s < NP - 1; ++s) {
      products(s, a1, b1);
      if (NP + s < NS) {
        put_one(NP + s, nbuf, live);
        fetch_one(NP + s, kt + 2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // tile t+1 complete in LDS; every wave is done reading tile t
    read_frags(nbuf, 0, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    products(NP - 1, a1, b1);
  }

  float rs[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) rs[i] = 0.f;
  if constexpr (RS) {
    constexpr int Q = BM / 4, R = NT / Q;
    static_assert(NT % Q == 0, "row-sum map");
    float4 t = rsq[0];
#pragma unroll
    for (int v = 1; v < SA::NV; ++v) {
      t.x = add_f32(t.x, rsq[v].x);
      t.y = add_f32(t.y, rsq[v].y);
      t.z = add_f32(t.z, rsq[v].z);
      t.w = add_f32(t.w, rsq[v].w);
    }
    __syncthreads();  // every wave is done with the LDS images
    float* part = smem;  // [R][BM]
    *reinterpret_cast<float4*>(part + (tid / Q) * BM + 4 * (tid % Q)) = t;
    __syncthreads();
    float* sums = smem + R * BM;  // [BM]
    if (tid < BM) {
      float s = part[tid];
      for (int r = 1; r < R; ++r) s += part[r * BM + tid];
      sums[tid] = s;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i) rs[i] = sums[wm0 + i * 32 + (lane & 31)];
    __syncthreads();  // the split-K hand-off reuses smem[0]
  }
  finish_tile32<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0, smem);
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
    float w[4];
    w[0] = apply_epilogue(p, row, col, p.alpha * acc.x, false);
    w[1] = apply_epilogue(p, row, col + 1, p.alpha * acc.y, false);
    w[2] = apply_epilogue(p, row, col + 2, p.alpha * acc.z, false);
    w[3] = apply_epilogue(p, row, col + 3, p.alpha * acc.w, false);
    if (p.Cp) store_planes_vec<4>(p, row, col, w);
  } else if (p.ones_col >= 0 && i - n4 < p.M) {
    const int64_t row = i - n4;
    const float* rsrc = p.part + (int64_t)S * MN + row;
    float acc = rsrc[0];
    for (int s = 1; s < S; ++s) acc += rsrc[(int64_t)s * p.M];
    apply_epilogue(p, row, p.ones_col, p.alpha * acc);
  }
}

// -------------------------------------------------- pre-split split-bf16 body (x6d) --
// The fp32 GEMM on the bf16 matrix core from operands that arrive ALREADY split into
// their (h, m, l) bf16 planes (dlrm_gemm_problem.a_planes / b_planes; the producing GEMM
// writes them in its epilogue, c_planes): no conversion in the main loop.  Plane panels
// go global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave instruction)
// through an S-stage ring, S - 1 K-tiles in flight; one barrier per 32-deep K-tile, the
// fragments of tile t+1 read under the second half of tile t's six products
// (v_mfma_f32_16x16x32_bf16: hh, hm, mh, hl, lh, mm; the map of pipe_body6).
// LDS images, one per plane and stage (bank maps checked offline for every fragment read:
// conflict-free):
//   KC  (MN x 32, k-contiguous):  16-B chunk c of row r in slot 4r + (c ^ ((r >> 1) & 3)),
//        fragments by ds_read_b128;
//   !KC (32 x MN, mn-contiguous): chunk c of k-row k in slot k(MN/8) + (c ^ f(k)),
//        f(k) = (MN/8 >= 16 ? 2 : 1)(k ^ (k >> 1)) mod MN/8, fragments by two
//        ds_read_b64_tr_b16 (hardware transpose).
// 4 stages: 144 KiB at 128x64, 96 KiB at 64x64 (one workgroup per CU).
template <int MN, bool KC>
struct PImg {
  static constexpr int SLOTS = 4 * MN;  // 16-B slots per plane and stage (MN x 32 bf16)
  static constexpr int BYTES = 16 * SLOTS;
  static constexpr int CPR = MN / 8;    // !KC: chunks per k-row
  static constexpr int BLK = SLOTS / 64;  // 1-KiB DMA blocks per plane
  __device__ __forceinline__ static int swk(int r) { return (r >> 1) & 3; }
  __device__ __forceinline__ static int swt(int k) {
    return ((CPR >= 16 ? 2 : 1) * (k ^ (k >> 1))) % CPR;
  }
  // (mn, k) of the 16-B chunk that fills slot `slot` (k: first of its 8 k, KC; the k-row, !KC)
  __device__ __forceinline__ static void src(int slot, int& mn, int& k) {
    if constexpr (KC) {
      const int r = slot >> 2;
      mn = r;
      k = 8 * ((slot & 3) ^ swk(r));
    } else {
      k = slot / CPR;
      mn = 8 * ((slot % CPR) ^ swt(k));
    }
  }
  // 8 bf16 along k of row / column mn0 + l16 (lane group kq holds k = 8kq .. 8kq+7)
  __device__ __forceinline__ static bf16x8 frag(const char* plane, int mn0, int l16, int kq) {
    if constexpr (KC) {
      const int r = mn0 + l16;
      return __builtin_bit_cast(
          bf16x8, *reinterpret_cast<const uint4*>(plane + 16 * (4 * r + (kq ^ swk(r)))));
    } else {
      const int q = l16 >> 2, pp = l16 & 3;
      const int ch = mn0 / 8 + (pp >> 1);
      const int k0 = 8 * kq + q, k1 = k0 + 4;
      const char* a0 = plane + 16 * (k0 * CPR + (ch ^ swt(k0))) + 8 * (pp & 1);
      const char* a1 = plane + 16 * (k1 * CPR + (ch ^ swt(k1))) + 8 * (pp & 1);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
      using s16x8 = __attribute__((ext_vector_type(8))) short;
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

template <int BM, int BN>
constexpr int x6d_stages() {
  return 4;  // (64x64 on 3 stages, two workgroups per CU: 20-45 % slower on the long-K
             //  wgrads, profiles/r03_x6p_dma_probe.txt)
}
template <int BM, int BN>
constexpr int x6d_smem_bytes() {
  return x6d_stages<BM, BN>() * 3 * 64 * (BM + BN);
}

// Sum of the 8 bf16 of a fragment (exact bf16 -> f32 widening, fixed order).
__device__ __forceinline__ float frag_sum(const bf16x8& f) {
  const uint4 u = __builtin_bit_cast(uint4, f);
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s = add_f32(s, __builtin_bit_cast(float, w[i] << 16));
    s = add_f32(s, __builtin_bit_cast(float, w[i] & 0xffff0000u));
  }
  return s;
}

// WGM x WGN waves (2x2: one wave per SIMD; 4x2: two, each on a 32x32 / 16x32 sub-tile, so a
// wave waiting on its DMA or LDS counters leaves the SIMD to its partner).  The plane
// images' 1-KiB DMA blocks (A's 3 planes, then B's, block b at LDS byte b * 1024 of the
// stage) are dealt round-robin over the waves: wave w issues blocks w, w + NW, ...
template <int BM, int BN, bool A_KC, bool B_KC, bool RS, int WGM = 2, int WGN = 2>
__device__ __forceinline__ void pipe_body_x6d(const GemmParams& p, int lb, char* smem) {
  constexpr int S = x6d_stages<BM, BN>();
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile");
  using IA = PImg<BM, A_KC>;
  using IB = PImg<BN, B_KC>;
  constexpr int STAGE = 3 * (IA::BYTES + IB::BYTES);
  constexpr int NBA = 3 * IA::BLK, NBB = 3 * IB::BLK, NB = NBA + NBB;
  constexpr int NI_LO = NB / NW, NI_HI = (NB + NW - 1) / NW, NREM = NB % NW;

  const int tile = lb / p.splits;
  const int split = lb - tile * p.splits;
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t K8 = (p.K + 7) / 8 * 8;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < K8) ? kbeg + p.kchunk : K8;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, l16 = lane & 15;
  const int wm0 = (wave / WGN) * WM, wn0 = (wave % WGN) * WN;
  const int nk = (int)((kend - kbeg + kBK - 1) / kBK);
  const bool hi = NREM == 0 || wave < NREM;  // this wave issues NI_HI blocks (else NI_LO)

  const int64_t a_ext = 2 * p.psa + (A_KC ? p.M * p.ldap : K8 * p.ldap);
  const int64_t b_ext = 2 * p.psb + (B_KC ? p.N * p.ldbp : K8 * p.ldbp);
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.Ap, (short)0, (int)(a_ext * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.Bp, (short)0, (int)(b_ext * 2), 0x00020000);
  // per DMA block of this wave: byte offset at the split's first K-tile (-1: row / column
  // outside the operand, or no such block) and the chunk's k within a K-tile
  int doff[NI_HI], dkp[NI_HI];
#pragma unroll
  for (int i = 0; i < NI_HI; ++i) {
    const int b = wave + NW * i;
    doff[i] = -1;
    dkp[i] = 0;
    if (b < NBA) {
      const int q = b / IA::BLK, bb = b - q * IA::BLK;
      int mn, k;
      IA::src(bb * 64 + lane, mn, k);
      const int64_t g = m0 + mn, gk = kbeg + k;
      doff[i] = g < p.M ? (int)(2 * (q * p.psa + (A_KC ? g * p.ldap + gk : gk * p.ldap + g)))
                        : -1;
      dkp[i] = k;
    } else if (b < NB) {
      const int q = (b - NBA) / IB::BLK, bb = (b - NBA) - q * IB::BLK;
      int mn, k;
      IB::src(bb * 64 + lane, mn, k);
      const int64_t g = n0 + mn, gk = kbeg + k;
      doff[i] = g < p.N ? (int)(2 * (q * p.psb + (B_KC ? g * p.ldbp + gk : gk * p.ldbp + g)))
                        : -1;
      dkp[i] = k;
    }
  }
  const int a_step = A_KC ? 2 * kBK : (int)(2 * kBK * p.ldap);
  const int b_step = B_KC ? 2 * kBK : (int)(2 * kBK * p.ldbp);
  const int krem = (int)(kend - kbeg);
  // DMA of K-tile t into stage t % S; chunks past the split's K range (and tiles t >= nk)
  // load zeros (out-of-descriptor offset); a wave's block count is fixed for the kernel
  auto issue = [&](int t) {
    char* st = smem + (t % S) * STAGE;
#pragma unroll
    for (int i = 0; i < NI_HI; ++i) {
      const int b = wave + NW * i;  // uniform
      if (i < NI_LO || hi) {
        const bool isa = b < NBA;
        const bool ok = doff[i] >= 0 && t * kBK + dkp[i] < krem;
        const int off = ok ? doff[i] + t * (isa ? a_step : b_step) : 0x7ffffff0;
        if (isa)
          dma16(ra, reinterpret_cast<const float*>(st + b * 1024), off);
        else
          dma16(rb, reinterpret_cast<const float*>(st + b * 1024), off);
      }
    }
  };
  auto wait_landed = [&](auto deep) {  // deep: tiles still allowed in flight after this one
    constexpr int D = decltype(deep)::value;
    if (hi)
      wait_vm<D * NI_HI>();
    else
      wait_vm<D * NI_LO>();
  };
  struct Frag {
    bf16x8 q[3];
  };
  auto read = [&](int t, Frag (&a)[FM], Frag (&b)[FN]) {
    const char* st = smem + (t % S) * STAGE;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i].q[q] = IA::frag(st + q * IA::BYTES, wm0 + i * 16, l16, kq);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j].q[q] = IB::frag(st + 3 * IA::BYTES + q * IB::BYTES, wn0 + j * 16, l16, kq);
    }
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rs[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) rs[i] = 0.f;
  auto products = [&](int s0, int s1, const Frag (&ca)[FM], const Frag (&cb)[FN]) {
    constexpr int PA[6] = {0, 2, 1, 0, 1, 0};  // (a, b) planes: hl, lh, mm, hm, mh, hh
    constexpr int PB[6] = {2, 0, 1, 1, 0, 0};
#pragma unroll
    for (int s = s0; s < s1; ++s)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[i].q[PA[s]], cb[j].q[PB[s]],
                                                              acc[i][j], 0, 0, 0);
  };
  auto rowsums = [&](const Frag (&ca)[FM]) {
    if constexpr (RS) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
        rs[i] = add_f32(rs[i], add_f32(add_f32(frag_sum(ca[i].q[0]), frag_sum(ca[i].q[1])),
                                       frag_sum(ca[i].q[2])));
    }
  };
  Frag ca[FM], cb[FN], na[FM], nb[FN];
#pragma unroll
  for (int t = 0; t < S - 1; ++t) issue(t);
  wait_landed(std::integral_constant<int, S - 2>());  // tile 0 landed (this wave)
  __builtin_amdgcn_s_barrier();  // (a bare barrier: __syncthreads' fence would drain the DMAs)
  asm volatile("" ::: "memory");
  read(0, ca, cb);
  auto step = [&](int t, const Frag (&a)[FM], const Frag (&b)[FN], Frag (&a2)[FM],
                  Frag (&b2)[FN]) {
    products(0, 3, a, b);
    wait_landed(std::integral_constant<int, S - 3>());  // tile t+1 landed (this wave)
    __builtin_amdgcn_s_barrier();  // every wave's has; every wave is done with tile t-1's stage
    asm volatile("" ::: "memory");
    issue(t + S - 1);  // into tile t-1's stage
    read(t + 1, a2, b2);
    products(3, 6, a, b);
    rowsums(a);
  };
  for (int t = 0; t < nk; t += 2) {
    step(t, ca, cb, na, nb);
    if (t + 1 >= nk) break;
    step(t + 1, na, nb, ca, cb);
  }
  wait_vm<0>();  // the trailing DMAs land before smem is reused or released
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
  }
  finish_tile<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0,
                                    reinterpret_cast<float*>(smem));
}

template <int BM, int BN>
constexpr int group_smem_floats() {
  // the largest LDS image over the four operand layouts (double-buffered A and B panels)
  return 2 * ((BM * (kBK + 4) > kBK * (BM + 4) ? BM * (kBK + 4) : kBK * (BM + 4)) +
              (BN * (kBK + 4) > kBK * (BN + 4) ? BN * (kBK + 4) : kBK * (BN + 4)));
}

// Body kinds: the four operand layouts, plus 4 = layout 2 (wgrad) with the row sums.
__host__ __device__ constexpr int kind_bit(int layout, bool rs) { return 1 << (rs ? 4 : layout); }

// Up to kMaxGroup independent problems; block -> (problem, tile, split) after the XCD remap.
// KINDS is the set of body kinds compiled in (a launch uses the smallest instantiation that
// covers its problems: fewer bodies, fewer registers).
template <int BM, int BN, int WGM, int WGN, int KINDS>
__global__ __launch_bounds__(WGM * WGN * 64, 2) void gemm_group_kernel(
    const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN>()];
  // Problems own consecutive PHYSICAL block ranges, so each one is dealt round-robin over
  // all eight XCDs (a remap across the whole launch would give each problem a few XCDs);
  // inside its range the XCD remap gives each XCD a contiguous run of that problem's tiles.
  const int b = blockIdx.x;
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
    if (kind == 0) return pipe_body<BM, BN, WGM, WGN, true, true, false>(p, lb, smem);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return pipe_body<BM, BN, WGM, WGN, true, false, false>(p, lb, smem);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return pipe_body<BM, BN, WGM, WGN, false, false, false>(p, lb, smem);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return pipe_body<BM, BN, WGM, WGN, false, true, false>(p, lb, smem);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return pipe_body<BM, BN, WGM, WGN, false, false, true>(p, lb, smem);
}

// The same grouped launch on the LDS-DMA body (pipe_body_dma).
template <int BM, int BN, int WGM, int WGN, int KINDS>
__global__ __launch_bounds__(WGM * WGN * 64, (BM * BN > 4096 ? 1 : 2)) void gemm_group_dma_kernel(
    const GemmGroup g) {
  constexpr int SM = dma_smem_floats<BM, BN>() > group_smem_floats<BM, BN>()
                         ? dma_smem_floats<BM, BN>()
                         : group_smem_floats<BM, BN>();
  __shared__ __attribute__((aligned(1024))) float smem[SM];
  const int b = blockIdx.x;
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
    if (kind == 0) return pipe_body_dma<BM, BN, WGM, WGN, true, true, false>(p, lb, smem);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return pipe_body_dma<BM, BN, WGM, WGN, true, false, false>(p, lb, smem);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return pipe_body_dma<BM, BN, WGM, WGN, false, false, false>(p, lb, smem);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return pipe_body_dma<BM, BN, WGM, WGN, false, true, false>(p, lb, smem);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return pipe_body_dma<BM, BN, WGM, WGN, false, false, true>(p, lb, smem);
}

// The same grouped launch on the split-bf16 body (pipe_body6).
template <int BM, int BN, int WGM, int WGN, int KINDS>
__global__ __launch_bounds__(WGM * WGN * 64, 2) void gemm_group6_kernel(const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[x6_smem_bytes<BM, BN>() / 4];
  const int b = blockIdx.x;
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
    if (kind == 0) return pipe_body6<BM, BN, WGM, WGN, true, true, false>(p, lb, smem);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return pipe_body6<BM, BN, WGM, WGN, true, false, false>(p, lb, smem);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return pipe_body6<BM, BN, WGM, WGN, false, false, false>(p, lb, smem);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return pipe_body6<BM, BN, WGM, WGN, false, true, false>(p, lb, smem);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return pipe_body6<BM, BN, WGM, WGN, false, false, true>(p, lb, smem);
}

// The same grouped launch on the 128x128 split-bf16 body (pipe_body6L): one wave per SIMD.
template <int BM, int BN, int WGM, int WGN, int KINDS>
__global__ __launch_bounds__(WGM * WGN * 64, 1) void gemm_group6L_kernel(const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[x6l_smem_bytes<BM, BN>() / 4];
  const int b = blockIdx.x;
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
    if (kind == 0) return pipe_body6L<BM, BN, WGM, WGN, true, true, false>(p, lb, smem);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return pipe_body6L<BM, BN, WGM, WGN, true, false, false>(p, lb, smem);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return pipe_body6L<BM, BN, WGM, WGN, false, false, false>(p, lb, smem);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return pipe_body6L<BM, BN, WGM, WGN, false, true, false>(p, lb, smem);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return pipe_body6L<BM, BN, WGM, WGN, false, false, true>(p, lb, smem);
}

// The same grouped launch on the pre-split body (pipe_body_x6d): LDS from the dynamic
// segment (96 or 144 KiB: one workgroup per CU).
template <int BM, int BN, int KINDS, int WGM = 2, int WGN = 2>
__global__ __launch_bounds__(WGM * WGN * 64, 1) void gemm_group6d_kernel(const GemmGroup g) {
  extern __shared__ __attribute__((aligned(1024))) char smem6d[];
  const int b = blockIdx.x;
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
    if (kind == 0) return pipe_body_x6d<BM, BN, true, true, false, WGM, WGN>(p, lb, smem6d);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return pipe_body_x6d<BM, BN, true, false, false, WGM, WGN>(p, lb, smem6d);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return pipe_body_x6d<BM, BN, false, false, false, WGM, WGN>(p, lb, smem6d);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return pipe_body_x6d<BM, BN, false, true, false, WGM, WGN>(p, lb, smem6d);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return pipe_body_x6d<BM, BN, false, false, true, WGM, WGN>(p, lb, smem6d);
}

// X [rows][cols] fp32 -> planes [3][rows][ldp] bf16, 8 elements per thread (columns
// [cols, ldp) untouched).
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ X,
                                                           int64_t rows, int64_t cols, int64_t ld,
                                                           __bf16* __restrict__ P, int64_t ldp,
                                                           int64_t ps) {
  const int64_t c8 = (cols + 7) / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * c8) return;
  const int64_t r = i / c8, c = 8 * (i - r * c8);
  __bf16* dst = P + r * ldp + c;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (c + u >= cols) break;
    const float v = X[r * ld + c + u];
    const __bf16 h = (__bf16)v;
    const float rr = v - (float)h;
    const __bf16 m = (__bf16)rr;
    dst[u] = h;
    dst[u + ps] = m;
    dst[u + 2 * ps] = (__bf16)(rr - (float)m);
  }
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

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

// Math of the pipelined GEMMs: exact-f32 MFMA, or the split-bf16 body where the plan table
// measured it faster and every GEMM of the launch agrees (default "auto"); DLRM_GEMM_MATH=
// f32 / x6 forces one everywhere.  Read per call, like the tuning overrides.
int gemm_math_env() {  // 0 f32, 1 x6 (64-wide tiles), 2 x6 on 128x128 tiles, -1 auto
  const char* v = getenv("DLRM_GEMM_MATH");
  if (v && strcmp(v, "x6") == 0) return 1;
  if (v && strcmp(v, "x6l") == 0) return 2;
  if (v && strcmp(v, "f32") == 0) return 0;
  return -1;
}

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
  const __bf16* Ap = nullptr;  // split-bf16 planes (dlrm_gemm_problem.a/b/c_planes)
  int64_t ldap = 0, psa = 0;
  const __bf16* Bp = nullptr;
  int64_t ldbp = 0, psb = 0;
  __bf16* Cp = nullptr;
  int64_t ldcp = 0, psc = 0;
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

// The pre-split body (pipe_body_x6d) takes a problem when both operands come with planes
// in whole 16-B chunks: pitches and plane strides % 8 (bf16), 16-B aligned bases, an
// mn-contiguous operand's extent % 8 and its K % 8 (its k-rows are read in 8-row chunks),
// 32-bit byte offsets.  DLRM_GEMM_PLANES=0 ignores the planes (A/B; read per call).
bool planes_ok(const Desc& d) {
  if (!d.Ap || !d.Bp || d.mode == DLRM_GEMM_REDUCE) return false;
  const char* v = getenv("DLRM_GEMM_PLANES");
  if (v && strcmp(v, "0") == 0) return false;
  const bool a_kc = !d.trans_a, b_kc = d.trans_b != 0;
  const int64_t K8 = (d.K + 7) / 8 * 8;
  auto ok = [&](const __bf16* P, int64_t ld, int64_t ps, bool kc, int64_t mn) {
    const int64_t ext = 2 * ps + (kc ? mn * ld : K8 * ld);
    return aligned16(P) && ld % 8 == 0 && ps % 8 == 0 && ps >= 0 &&
           (kc ? ld >= K8 : (mn % 8 == 0 && d.K % 8 == 0 && ld >= mn)) &&
           ext * 2 < 0x7ff00000LL;
  };
  return d.K > 0 && ok(d.Ap, d.ldap, d.psa, a_kc, d.M) && ok(d.Bp, d.ldbp, d.psb, b_kc, d.N);
}

struct PlanEntry {
  int64_t M, N, K;
  int layout, bm, bn, split;
  int wm = 2, wn = 2;
  int x6 = 0;   // 1: the split-bf16 body measured faster (tools/gemm_x6_ab.py); 2: on
                //    128x128 tiles (pipe_body6L)
  int dma = 0;  // 1: the LDS-DMA f32 body (tools/gemm_body_ab.py)
};

// Measured plans for the DLRM step shapes of single-problem launches (exact match), from
// tools/gemm_sweep.py on MI355X.
constexpr PlanEntry kPlans[] = {
#include "gemm_plans.inc"
    {0, 0, 0, 0, 64, 64, 1},  // sentinel (never matches: M = 0)
};

// Compiled tiles (BM x BN on 2x2 waves): 64x64, 128x64, 64x128, 32x64, 64x32.  (Other
// wave layouts of pipe_body - 64x32 on 2x1, 32x64 on 1x2, 128x32 on 4x1 - measured slower
// on every DLRM shape: tools/gemm_cfg_ab.py, profiles/r02_gemm_cfg_ab.txt.)
bool tile_ok(int bm, int bn, int wm, int wn) {
  return wm == 2 && wn == 2 &&
         ((bm == 64 && bn == 64) || (bm == 128 && bn == 64) || (bm == 64 && bn == 128) ||
          (bm == 32 && bn == 64) || (bm == 64 && bn == 32));
}

struct Tile {
  int bm = 64, bn = 32, wm = 2, wn = 2;
  int x6 = 0;   // math vote of a problem / the launch's math (3: pre-split planes, x6d)
  int dma = 0;  // f32 body vote of a problem / the launch's body (1: LDS-DMA)
  bool operator==(const Tile& o) const {
    return bm == o.bm && bn == o.bn && wm == o.wm && wn == o.wn;
  }
};

// Plan of ONE problem, independent of what it is grouped with (so a problem's result is
// bitwise the same in any group: the split decides the summation order, the tile shape
// does not).  Tuning overrides (read per call, for sweeps): DLRM_GEMM_CFG=<BM>x<BN> or
// <BM>x<BN>x<WGM>x<WGN>, DLRM_GEMM_SPLIT=<n>.
// A/B override for the large shapes (>= 2^20 outputs): DLRM_GEMM_BIG=dma64 puts them on
// 64x64 tiles and the LDS-DMA body; dma64h also halves a split K (read per call).
void big_override(const Desc& d, Tile& t, Plan& pl) {
  const char* v = getenv("DLRM_GEMM_BIG");
  if (!v || strncmp(v, "dma64", 5) != 0 || d.M * d.N < (1 << 20)) return;
  t = Tile{64, 64, 2, 2, 0, 1};
  if (v[5] == 'h' && pl.splits > 1) pl = make_plan(pl.splits / 2, d.K);
}

// DLRM_GEMM_MATH=x6l: every problem of >= 2^18 outputs on the 128x128 split-bf16 body,
// K split until the tiles fill the CUs once (>= 256 blocks, K chunks >= 128).  The split is
// decided here, per problem, so a problem sums in the same order in any launch.
void x6l_override(const Desc& d, Tile& t, Plan& pl) {
  if (gemm_math_env() != 2 || d.M * d.N < (1 << 18)) return;
  t = Tile{128, 128, 2, 2, 2};
  const int force_split = env_int("DLRM_GEMM_SPLIT", 0);  // (A/B sweeps)
  if (force_split > 0) {
    pl = make_plan(force_split, d.K);
    return;
  }
  const int64_t tiles = dlrm::ceil_div(d.M, 128) * dlrm::ceil_div(d.N, 128);
  int64_t s = 1;
  while (tiles * s < 256 && dlrm::ceil_div(d.K, s + 1) >= 128 && s < kMaxSplit) ++s;
  pl = make_plan(s, d.K);
}

// Pre-split problems: 128x64 tiles when they fill the CUs once (>= 240 tiles), else 64x64;
// K split until >= 256 blocks with K chunks >= 256 (PARTIAL: the caller's count, if any).
void plan_x6d(const Desc& d, Tile& t, Plan& pl) {
  const int64_t t128 = dlrm::ceil_div(d.M, 128) * dlrm::ceil_div(d.N, 64);
  t = t128 >= 240 ? Tile{128, 64, 2, 2, 3} : Tile{64, 64, 2, 2, 3};
  if (d.mode == DLRM_GEMM_PARTIAL && d.splits > 0) {
    pl = make_plan(d.splits, d.K);
    return;
  }
  const int force_split = env_int("DLRM_GEMM_SPLIT", 0);  // (A/B sweeps)
  if (force_split > 0) {
    pl = make_plan(force_split, d.K);
    return;
  }
  const int64_t tiles = dlrm::ceil_div(d.M, t.bm) * dlrm::ceil_div(d.N, t.bn);
  int64_t s = 1;
  while (tiles * s < 256 && dlrm::ceil_div(d.K, s + 1) >= 256 && s < kMaxSplit) ++s;
  pl = make_plan(s, d.K);
}

void plan_one(const Desc& d, Tile& t, Plan& pl) {
  t = Tile{64, 64, 2, 2};
  if (d.mode == DLRM_GEMM_REDUCE) {  // elementwise job: no tiles, no K
    pl.splits = d.splits;
    pl.kchunk = 0;
    return;
  }
  if (planes_ok(d)) return plan_x6d(d, t, pl);
  if (d.mode == DLRM_GEMM_PARTIAL && d.splits > 0) {  // caller-sized partial buffer
    Desc q = d;
    q.mode = DLRM_GEMM_FULL;
    plan_one(q, t, pl);
    pl = make_plan(d.splits, d.K);
    return;
  }
  const char* cfg = getenv("DLRM_GEMM_CFG");
  const int force_split = env_int("DLRM_GEMM_SPLIT", 0);
  if (cfg && *cfg) {
    int a = 64, b = 64, wm = 2, wn = 2;
    const int got = sscanf(cfg, "%dx%dx%dx%d", &a, &b, &wm, &wn);
    if (got == 2) wm = wn = 2;
    if (got >= 2 && tile_ok(a, b, wm, wn)) t = Tile{a, b, wm, wn};
    pl = make_plan(force_split > 0 ? force_split : 1, d.K);
    return;
  }
  if (!getenv("DLRM_GEMM_NOTABLE"))
    for (const PlanEntry& e : kPlans)
      if (e.M == d.M && e.N == d.N && e.K == d.K && e.layout == layout_of(d)) {
        t = Tile{e.bm, e.bn, e.wm, e.wn, e.x6, e.dma};
        pl = make_plan(e.split, d.K);
        if (e.x6 != 2) x6l_override(d, t, pl);
        big_override(d, t, pl);
        return;
      }
  // Heuristic (shapes not in the table): 64x32 tiles (the sweep's best almost everywhere);
  // FULL problems run unsplit unless they have fewer than one tile per CU (an in-launch
  // split costs a hand-off); PARTIAL ones split K until >= 2 blocks per CU, every K chunk
  // >= 256 (8 K-tiles).
  t = Tile{64, 32, 2, 2};
  const int64_t tiles = dlrm::ceil_div(d.M, 64) * dlrm::ceil_div(d.N, 32);
  const int target = env_int("DLRM_GEMM_TARGET", d.mode == DLRM_GEMM_PARTIAL ? 512 : 256);
  int64_t s = 1;
  while (tiles * s < target && dlrm::ceil_div(d.K, s + 1) >= 256 && s < kMaxSplit) ++s;
  pl = make_plan(s, d.K);
  x6l_override(d, t, pl);
  big_override(d, t, pl);
}

// Tile config of a launch: the GEMM problems' common choice, else 64x32 (REDUCE jobs have
// no tiles and do not vote).
void plan_launch(int n, const Desc* d, Tile& t, Plan* pl) {
  bool first = true;
  t = Tile{64, 64, 2, 2};
  int votes = 0, gemms = 0, dvotes = 0, lvotes = 0, pvotes = 0;
  for (int i = 0; i < n; ++i) {
    Tile a;
    plan_one(d[i], a, pl[i]);
    if (d[i].mode == DLRM_GEMM_REDUCE) continue;
    ++gemms;
    votes += a.x6 == 1;
    lvotes += a.x6 == 2;
    pvotes += a.x6 == 3;
    dvotes += a.dma;
    if (first) {
      t = a;
      first = false;
    } else if (!(a == t)) {
      t = Tile{64, 32, 2, 2};
    }
  }
  if (gemms > 0 && pvotes == gemms) {  // every GEMM has planes: the pre-split body
    t.x6 = 3;
    if (!(t.bm == 128 && t.bn == 64)) t = Tile{64, 64, 2, 2, 3};
    return;
  }
  if (pvotes > 0)  // mixed: the f32 body for all (pre-split problems re-planned for it)
    for (int i = 0; i < n; ++i)
      if (d[i].mode != DLRM_GEMM_REDUCE && planes_ok(d[i])) {
        Desc q = d[i];
        q.Ap = q.Bp = nullptr;
        Tile a;
        Plan keep = pl[i];
        plan_one(q, a, pl[i]);
        if (d[i].mode == DLRM_GEMM_PARTIAL) pl[i] = keep;  // the REDUCE repeats this count
      }
  const int env = gemm_math_env();
  // 128x128 split-bf16 only when every GEMM of the launch asks for it (their tiles agree)
  t.x6 = gemms > 0 && lvotes == gemms ? 2 : env == 1 ? 1 : env == 0 ? 0
         : (gemms > 0 && votes == gemms);
  t.dma = gemms > 0 && dvotes == gemms;  // every GEMM of the launch asks for the DMA body
  if (t.x6 == 1 && (t.bm == 128 || t.bn == 128)) t = Tile{64, 64, 2, 2, 1};
  if (t.x6 != 2 && t.bm == 128 && t.bn == 128) t = Tile{64, 32, 2, 2, t.x6, t.dma};
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

// Body of a launch: kBodyReg (register-staged f32 pipe_body), kBodyX6 (split-bf16),
// kBodyDma (LDS-DMA f32 pipe_body_dma, where the plan asks for it).
constexpr int kBodyReg = 0, kBodyX6 = 1, kBodyDma = 2, kBodyX6L = 3, kBodyX6D = 4;

// f32 body of a launch: the plan's vote, or DLRM_GEMM_BODY=reg / dma everywhere (A/B; read
// per call).
int f32_body(int plan_dma) {
  const char* v = getenv("DLRM_GEMM_BODY");
  if (v && strcmp(v, "reg") == 0) return kBodyReg;
  if (v && strcmp(v, "dma") == 0) return kBodyDma;
  return plan_dma ? kBodyDma : kBodyReg;
}

// The x6d kernels' dynamic LDS (> 64 KiB) must be opted into once per kernel and DEVICE
// (`mask`: one bit per device ordinal; idempotent, so a benign race between host threads).
inline int x6d_smem_optin(const void* fn, int bytes, unsigned long long& mask) {
  int dev = 0;
  DLRM_HIP_CALL(hipGetDevice(&dev), "dlrm_gemm_f32 (x6d)");
  const unsigned long long bit = dev < 64 ? (1ull << dev) : 0ull;
  if (bit && (mask & bit)) return DLRM_OK;
  DLRM_HIP_CALL(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes),
                "dlrm_gemm_f32 (x6d)");
  mask |= bit;
  return DLRM_OK;
}

template <int BM, int BN, int WGM, int WGN>
int launch_x6d_all(const GemmGroup& g, hipStream_t st) {
  constexpr int SM = x6d_smem_bytes<BM, BN>();
  static unsigned long long mask = 0;
  const int rc = x6d_smem_optin((const void*)gemm_group6d_kernel<BM, BN, 31, WGM, WGN>, SM, mask);
  if (rc != DLRM_OK) return rc;
  hipLaunchKernelGGL((gemm_group6d_kernel<BM, BN, 31, WGM, WGN>), dim3(g.total),
                     dim3(WGM * WGN * 64), SM, st, g);
  DLRM_LAUNCH_CHECK("dlrm_gemm_f32 (x6d)");
  return DLRM_OK;
}

template <int BM, int BN, int BODY = kBodyDma, int WGM = 2, int WGN = 2>
int launch_group(int n, const Desc* d, const Plan* pl, void* ws, size_t ws_bytes, hipStream_t st) {
  constexpr int NT = WGM * WGN * 64;
  GemmGroup g{};
  g.n = n;
  const int pub = env_int("DLRM_GEMM_PUB", 1);
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
    p.pub = pub;
    p.mode = d[i].mode;
    p.part = d[i].part;
    p.Ap = d[i].Ap, p.ldap = d[i].ldap, p.psa = d[i].psa;
    p.Bp = d[i].Bp, p.ldbp = d[i].ldbp, p.psb = d[i].psb;
    p.Cp = d[i].Cp, p.ldcp = d[i].ldcp, p.psc = d[i].psc;
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
  const dim3 grid(g.total), block(NT);
  // instantiations: every single kind, the MLP-backward pairs (dgrad + wgrad with / without
  // row sums, two wgrads), else all kinds
  if constexpr (BODY == kBodyX6D) {
    constexpr int SM = x6d_smem_bytes<BM, BN>();
#define K_(M_)                                                                              \
  case M_: {                                                                               \
    static unsigned long long mask = 0;                                                    \
    const int rc =                                                                         \
        x6d_smem_optin((const void*)gemm_group6d_kernel<BM, BN, M_, WGM, WGN>, SM, mask);  \
    if (rc != DLRM_OK) return rc;                                                          \
    hipLaunchKernelGGL((gemm_group6d_kernel<BM, BN, M_, WGM, WGN>), grid, block, SM, st, g); \
    break;                                                                                 \
  }
    switch (kinds) {
      K_(0) K_(1) K_(2) K_(4) K_(16) K_(2 | 16) K_(2 | 4)
      default:
        return launch_x6d_all<BM, BN, WGM, WGN>(g, st);
    }
#undef K_
  } else if constexpr (BODY == kBodyX6L) {
    switch (kinds) {
#define K_(M_)                                                                            \
  case M_:                                                                               \
    hipLaunchKernelGGL((gemm_group6L_kernel<BM, BN, WGM, WGN, M_>), grid, block, 0, st, g); \
    break;
      K_(0) K_(1) K_(2) K_(4) K_(8) K_(16) K_(2 | 16) K_(2 | 4) K_(4 | 16)
#undef K_
      default:
        hipLaunchKernelGGL((gemm_group6L_kernel<BM, BN, WGM, WGN, 31>), grid, block, 0, st, g);
    }
  } else if constexpr (BODY == kBodyX6) {
    switch (kinds) {
#define K_(M_)                                                                           \
  case M_:                                                                              \
    hipLaunchKernelGGL((gemm_group6_kernel<BM, BN, WGM, WGN, M_>), grid, block, 0, st, g); \
    break;
      K_(0) K_(1) K_(2) K_(4) K_(8) K_(16) K_(2 | 16) K_(2 | 4) K_(4 | 16)
#undef K_
      default:
        hipLaunchKernelGGL((gemm_group6_kernel<BM, BN, WGM, WGN, 31>), grid, block, 0, st, g);
    }
  } else if constexpr (BODY == kBodyDma) {
    switch (kinds) {
#define K_(M_)                                                                              \
  case M_:                                                                                 \
    hipLaunchKernelGGL((gemm_group_dma_kernel<BM, BN, WGM, WGN, M_>), grid, block, 0, st, g); \
    break;
      K_(0) K_(1) K_(2) K_(4) K_(8) K_(16) K_(2 | 16) K_(2 | 4) K_(4 | 16)
#undef K_
      default:
        hipLaunchKernelGGL((gemm_group_dma_kernel<BM, BN, WGM, WGN, 31>), grid, block, 0, st, g);
    }
  } else {
    switch (kinds) {
#define K_(M_)                                                                          \
  case M_:                                                                             \
    hipLaunchKernelGGL((gemm_group_kernel<BM, BN, WGM, WGN, M_>), grid, block, 0, st, g); \
    break;
      K_(0) K_(1) K_(2) K_(4) K_(8) K_(16) K_(2 | 16) K_(2 | 4) K_(4 | 16)
#undef K_
      default:
        hipLaunchKernelGGL((gemm_group_kernel<BM, BN, WGM, WGN, 31>), grid, block, 0, st, g);
    }
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
  p.Cp = d.Cp, p.ldcp = d.ldcp, p.psc = d.psc;  // (c_planes are kept on every path)
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
  DLRM_ARG(!d.Cp || (d.ldcp >= d.ldc && d.psc >= 0 && d.ldcp % 8 == 0 && d.psc % 8 == 0 &&
                     aligned16(d.Cp)),
           "dlrm_gemm_f32: c_planes need 16-B aligned planes, ldc_planes >= ldc, "
           "ldc_planes and plane_stride %% 8 == 0");
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
  return group_ws_bytes(m, q, t, pl);
}

int run(int n, const Desc* d, void* ws, size_t ws_bytes, hipStream_t st) {
  DLRM_ARG(n >= 1 && n <= kMaxGroup, "dlrm_gemm_f32_group: 1..%d problems", kMaxGroup);
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
  if (m == 0) return DLRM_OK;
  Tile t;
  Plan pl[kMaxGroup];
  plan_launch(m, q, t, pl);
  const size_t need = group_ws_bytes(m, q, t, pl);
  if (need > 0 && (!ws || ws_bytes < need)) {  // no workspace: in-launch splits off
    // (PARTIAL / REDUCE plans pair with each other across launches: kept)
    for (int i = 0; i < m; ++i)
      if (q[i].mode == DLRM_GEMM_FULL) pl[i] = make_plan(1, q[i].K);
  }
  if (t.x6 == 3) {  // pre-split planes
    // 4x2 waves (two per SIMD) by default; DLRM_X6D_WAVES=4: the 2x2 layout (A/B)
    if (env_int("DLRM_X6D_WAVES", 8) == 4) {
      if (t.bm == 128) return launch_group<128, 64, kBodyX6D>(m, q, pl, ws, ws_bytes, st);
      return launch_group<64, 64, kBodyX6D>(m, q, pl, ws, ws_bytes, st);
    }
    if (t.bm == 128) return launch_group<128, 64, kBodyX6D, 4, 2>(m, q, pl, ws, ws_bytes, st);
    return launch_group<64, 64, kBodyX6D, 4, 2>(m, q, pl, ws, ws_bytes, st);
  }
  // 128x128 split-bf16 on 2x4 waves (64x32 per wave, two waves per SIMD; the 2x2 layout,
  // one wave per SIMD, measured 1.15x slower: profiles/r03_x6l_ab.txt)
  if (t.x6 == 2) return launch_group<128, 128, kBodyX6L, 2, 4>(m, q, pl, ws, ws_bytes, st);
  if (t.x6) {  // split-bf16 body: 128-wide tiles stage too much per K-tile (and 128x128 on
              // 8-wave workgroups leaves half the CUs idle at M = 2048: r03_gemm_tiles_ab.txt)
    if (t.bm == 32) return launch_group<32, 64, kBodyX6>(m, q, pl, ws, ws_bytes, st);
    if (t.bn == 32) return launch_group<64, 32, kBodyX6>(m, q, pl, ws, ws_bytes, st);
    return launch_group<64, 64, kBodyX6>(m, q, pl, ws, ws_bytes, st);
  }
  if (f32_body(t.dma) == kBodyReg) {
    if (t.bm == 128) return launch_group<128, 64, kBodyReg>(m, q, pl, ws, ws_bytes, st);
    if (t.bn == 128) return launch_group<64, 128, kBodyReg>(m, q, pl, ws, ws_bytes, st);
    if (t.bm == 32) return launch_group<32, 64, kBodyReg>(m, q, pl, ws, ws_bytes, st);
    if (t.bn == 32) return launch_group<64, 32, kBodyReg>(m, q, pl, ws, ws_bytes, st);
    return launch_group<64, 64, kBodyReg>(m, q, pl, ws, ws_bytes, st);
  }
  if (t.bm == 128) return launch_group<128, 64>(m, q, pl, ws, ws_bytes, st);
  if (t.bn == 128) return launch_group<64, 128>(m, q, pl, ws, ws_bytes, st);
  if (t.bm == 32) return launch_group<32, 64>(m, q, pl, ws, ws_bytes, st);
  if (t.bn == 32) return launch_group<64, 32>(m, q, pl, ws, ws_bytes, st);
  return launch_group<64, 64>(m, q, pl, ws, ws_bytes, st);
}

Desc desc_of(const dlrm_gemm_problem& g) {
  Desc d;
  d.trans_a = g.trans_a, d.trans_b = g.trans_b;
  d.M = g.M, d.N = g.N, d.K = g.K, d.alpha = g.alpha;
  d.A = g.A, d.lda = g.lda, d.B = g.B, d.ldb = g.ldb;
  d.C = g.C, d.ldc = g.ldc, d.epi = g.epilogue, d.bias = g.bias;
  d.aux = g.aux, d.ldaux = g.ld_aux, d.ones_col = g.ones_col;
  d.mode = g.mode, d.splits = g.splits, d.part = g.partial;
  d.Ap = static_cast<const __bf16*>(g.a_planes), d.ldap = g.lda_planes, d.psa = g.a_plane_stride;
  d.Bp = static_cast<const __bf16*>(g.b_planes), d.ldbp = g.ldb_planes, d.psb = g.b_plane_stride;
  d.Cp = static_cast<__bf16*>(g.c_planes), d.ldcp = g.ldc_planes, d.psc = g.c_plane_stride;
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

extern "C" int dlrm_split_planes(const float* X, int64_t rows, int64_t cols, int64_t ld,
                                 void* planes, int64_t ld_planes, int64_t plane_stride,
                                 dlrm_stream_t stream) {
  DLRM_ARG(rows >= 0 && cols >= 0 && ld >= cols && ld_planes % 8 == 0 && ld_planes >= cols &&
               plane_stride >= 0,
           "dlrm_split_planes: bad sizes");
  const int64_t n = rows * ((cols + 7) / 8);
  if (n == 0) return DLRM_OK;
  DLRM_ARG(X && planes, "dlrm_split_planes: null pointer");
  hipLaunchKernelGGL(split_planes_kernel, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), X, rows, cols, ld, static_cast<__bf16*>(planes),
                     ld_planes, plane_stride);
  DLRM_LAUNCH_CHECK("dlrm_split_planes");
  return DLRM_OK;
}
