// Exact-fp32 GEMM with fused epilogues on the gfx950 fp32 matrix core
// (v_mfma_f32_32x32x2_f32: 64 FLOP/clk/SIMD, k-ordered fmaf chain, no xf32).
//
// Serves the DLRM MLPs (DLRM_Net.create_mlp / apply_mlp, dlrm_s_pytorch.py:227-265,
// 518-524): Linear forward with bias(+ReLU) fused, dgrad with the ReLU mask of the
// previous activation fused, wgrad with the SGD update fused (single GPU) or stored
// into the flat gradient bucket (multi GPU, all-reduced before the update).
//
// Structure: 256-thread workgroups = 4 waves in a 2x2 arrangement, each wave owning a
// (BM/2)x(BN/2) sub-tile of 32x32 MFMA accumulators (16 AGPRs each).  K is staged
// BK deep through double-buffered LDS.  The k-order inside a K-tile is permuted so
// that a lane's operands are CONTIGUOUS: lane (l, h) (l = lane & 31, h = lane >> 5)
// feeds k = h*BK/2 + s at MFMA step s, for both operands, so
//   * an operand that is k-contiguous in HBM (X rows, nn.Linear W rows) is staged
//     [mn][k] with float4 loads + ds_write_b128 and its fragments are ds_read_b128
//     (16 k-values in 4 instructions);
//   * an mn-contiguous operand is staged [k][mn] (float4 along mn, ds_write_b128) and
//     read with conflict-free ds_read_b32 (32 consecutive floats per half-wave).
// The next K-tile is fetched into registers before the MFMAs of the current one and
// written after them (one barrier per K-tile).  Workgroups are remapped bijectively
// so each XCD (private 4 MiB L2) receives a contiguous run of output tiles.
//
// DLRM's GEMMs are small for 256 CUs (M = batch <= 2048, N,K <= 1024) and the weight
// gradients have a long K (= the batch) over a small M x N: the planner may split K;
// split partials go to a caller workspace and a reduce kernel sums them IN SPLIT ORDER
// (deterministic) and applies the epilogue.  Tile / BK / split per shape come from
// on-device sweeps (tools/gemm_sweep.py), with a heuristic for other shapes.
#include <cstdlib>
#include <cstring>

#include "common.hpp"

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kThreads = 256;
constexpr int kMaxSplit = 32;
constexpr int kMinSplitK = 128;

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
  int tiles_m, tiles_n;
  int64_t kchunk;  // K range per split (multiple of BK)
  float* ws;       // split partials [splits][M][N] (splits > 1 only)
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

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // Contiguous tile runs per XCD (blocks b and b+8 share an XCD); bijective for any nwg.
  const int xcd = bid % 8;
  const int q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// C = epilogue(v) where v = alpha * acc (already scaled).
__device__ __forceinline__ void apply_epilogue(const GemmParams& p, int64_t row, int64_t col,
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
}

// KS = 1: 4 waves (2x2) share the K-tile.  KS = 2: 8 waves, two k-groups of 4; group g
// takes k in [g*BK/2, (g+1)*BK/2) of every K-tile (twice the waves per SIMD for the
// same output tile, no extra global traffic) and the groups' accumulators are summed
// through LDS in group order before the epilogue.
template <int BM, int BN, int BKT, int KS, bool A_KC, bool B_KC, bool VEC>
__global__ __launch_bounds__(kThreads * KS, (BM * BN * KS >= 128 * 128 * 2 || BKT >= 64) ? 1 : 2)
void gemm_f32_mfma_kernel(GemmParams p) {
  constexpr int NT = kThreads * KS;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int KW = BKT / KS;   // k per wave per K-tile
  constexpr int NSTEP = KW / 2;  // MFMA k-steps per wave per K-tile
  constexpr int CH = NSTEP < 16 ? NSTEP : 16;
  using SA = Stage<BM, BKT, A_KC, VEC, NT>;
  using SB = Stage<BN, BKT, B_KC, VEC, NT>;
  static_assert(KS == 1 || 2 * (SA::SIZE + SB::SIZE) >= BM * BN, "LDS too small for k-group sum");
  __shared__ __attribute__((aligned(16))) float smem[2 * (SA::SIZE + SB::SIZE)];
  float* As0 = smem;
  float* Bs0 = smem + SA::SIZE;
  float* As1 = smem + SA::SIZE + SB::SIZE;
  float* Bs1 = As1 + SA::SIZE;

  const int nwg = p.tiles_m * p.tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / p.tiles_n;
  const int tn = wg - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int split = blockIdx.y;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int kg = wave >> 2;  // k-group
  const int wq = wave & 3;
  const int lane = tid & 63;
  const int h = lane >> 5;
  const int l32 = lane & 31;
  const int wm0 = (wq >> 1) * WM;
  const int wn0 = (wq & 1) * WN;

  // A single 32x32 accumulator per wave would be one dependent MFMA chain (64-cycle
  // issue == 64-cycle accumulate latency: any bubble stalls the wave); such waves
  // alternate two chains over the k-steps and add them at the end.
  constexpr int NCH = (TM * TN >= 2) ? 1 : 2;
  f32x16 acc[TM][TN], acc2[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = acc2[i][j][r] = 0.f;

  SA sa;
  SB sb;
  const int64_t nk = (kend - kbeg + BKT - 1) / BKT;
  if (nk > 0) {
    sa.load(p.A, p.lda, m0, p.M, kbeg, kend, tid);
    sb.load(p.B, p.ldb, n0, p.N, kbeg, kend, tid);
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
      sa.load(p.A, p.lda, m0, p.M, kbeg + (kt + 1) * BKT, kend, tid);
      sb.load(p.B, p.ldb, n0, p.N, kbeg + (kt + 1) * BKT, kend, tid);
    }
#pragma unroll
    for (int sub = 0; sub < NSTEP / CH; ++sub) {
      const int kbase = kg * KW + h * NSTEP + sub * CH;
      float a[TM][CH], b[TN][CH];
#pragma unroll
      for (int i = 0; i < TM; ++i) sa.template frag<CH>(As, wm0 + i * 32, l32, kbase, a[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) sb.template frag<CH>(Bs, wn0 + j * 32, l32, kbase, b[j]);
#pragma unroll
      for (int s = 0; s < CH; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if (NCH == 2 && (s & 1))
              acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], acc2[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
          }
    }
    if (more) {
      sa.store(odd ? As0 : As1, tid);
      sb.store(odd ? Bs0 : Bs1, tid);
    }
    __syncthreads();
  }

  if constexpr (NCH == 2) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += acc2[i][j];
  }
  if constexpr (KS == 2) {
    // group 1 hands its accumulators to group 0 through LDS (free after the last barrier)
    float* red = smem + (size_t)wq * (WM * WN);
    if (kg == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[((i * TN + j) * 16 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (kg == 1) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] += red[((i * TN + j) * 16 + r) * 64 + lane];
  }

  // Epilogue: accumulator register r of a 32x32 tile holds
  //   row (r&3) + 8*(r>>2) + 4*(lane>>5), column lane&31.
  const bool partial = gridDim.y > 1;
  float* wsp = partial ? p.ws + (int64_t)split * p.M * p.N : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = n0 + wn0 + j * 32 + l32;
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        if (partial)
          wsp[row * p.N + col] = acc[i][j][r];
        else
          apply_epilogue(p, row, col, p.alpha * acc[i][j][r]);
      }
    }
  }
}

// 16x16x4 variant: v_mfma_f32_16x16x4_f32 (32-cycle issue, 40-cycle accumulate latency)
// with FM x FN independent 16x16 accumulators per wave, so a single wave per SIMD keeps
// the matrix pipe busy.  Lane l feeds row/col l & 15 and k = (l >> 4) * BK/4 + s at
// step s (BK/4 contiguous k per lane: two ds_read_b128 per k-contiguous fragment).
template <int BM, int BN, bool A_KC, bool B_KC, bool VEC>
__global__ __launch_bounds__(kThreads, 2) void gemm_f32_mfma16_kernel(GemmParams p) {
  constexpr int BKT = 32;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int KL = BKT / 4;
  using SA = Stage<BM, BKT, A_KC, VEC, kThreads>;
  using SB = Stage<BN, BKT, B_KC, VEC, kThreads>;
  __shared__ __attribute__((aligned(16))) float smem[2 * (SA::SIZE + SB::SIZE)];
  float* As0 = smem;
  float* Bs0 = smem + SA::SIZE;
  float* As1 = smem + SA::SIZE + SB::SIZE;
  float* Bs1 = As1 + SA::SIZE;

  const int nwg = p.tiles_m * p.tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / p.tiles_n;
  const int tn = wg - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int split = blockIdx.y;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int kq = lane >> 4;
  const int l16 = lane & 15;
  const int wm0 = (wave >> 1) * WM;
  const int wn0 = (wave & 1) * WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Two-deep register ring: tile t+2 is in flight while tile t is multiplied and tile
  // t+1 is written to LDS, so each global load has two MFMA blocks to arrive.
  const int64_t nk = (kend - kbeg + BKT - 1) / BKT;
  SA ra0, ra1;
  SB rb0, rb1;
  auto fetch = [&](SA& ra, SB& rb, int64_t t) {
    if (t < nk) {
      ra.load(p.A, p.lda, m0, p.M, kbeg + t * BKT, kend, tid);
      rb.load(p.B, p.ldb, n0, p.N, kbeg + t * BKT, kend, tid);
    }
  };
  auto compute = [&](const float* As, const float* Bs) {
    float a[FM][KL], b[FN][KL];
#pragma unroll
    for (int i = 0; i < FM; ++i) ra0.template frag<KL>(As, wm0 + i * 16, l16, kq * KL, a[i]);
#pragma unroll
    for (int j = 0; j < FN; ++j) rb0.template frag<KL>(Bs, wn0 + j * 16, l16, kq * KL, b[j]);
#pragma unroll
    for (int s = 0; s < KL; ++s)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  };
  fetch(ra0, rb0, 0);
  fetch(ra1, rb1, 1);
  if (nk > 0) {
    ra0.store(As0, tid);
    rb0.store(Bs0, tid);
  }
  fetch(ra0, rb0, 2);
  __syncthreads();
  for (int64_t kt = 0; kt < nk; kt += 2) {
    compute(As0, Bs0);
    if (kt + 1 < nk) {
      ra1.store(As1, tid);
      rb1.store(Bs1, tid);
    }
    fetch(ra1, rb1, kt + 3);
    __syncthreads();
    if (kt + 1 >= nk) break;
    compute(As1, Bs1);
    if (kt + 2 < nk) {
      ra0.store(As0, tid);
      rb0.store(Bs0, tid);
    }
    fetch(ra0, rb0, kt + 4);
    __syncthreads();
  }

  // Epilogue: register r of a 16x16 accumulator holds row 4*(lane>>4) + r, col lane&15.
  const bool partial = gridDim.y > 1;
  float* wsp = partial ? p.ws + (int64_t)split * p.M * p.N : nullptr;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = n0 + wn0 + j * 16 + l16;
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm0 + i * 16 + 4 * kq + r;
        if (row >= p.M) continue;
        if (partial)
          wsp[row * p.N + col] = acc[i][j][r];
        else
          apply_epilogue(p, row, col, p.alpha * acc[i][j][r]);
      }
    }
  }
}

// Software-pipelined 16x16x4 kernel (one barrier per K-tile, MFMAs kept dense):
//   * the fragments of K-tile t are in registers before its MFMAs start (read from LDS
//     at the end of iteration t-1, under the last MFMA step);
//   * during the MFMAs of tile t, the staged registers of tile t+1 (fetched from HBM one
//     iteration earlier) are written to the other LDS buffer one float4 per k-step, and
//     each freed register is immediately refilled with tile t+2's float4;
//   * one barrier, then tile t+1's fragments are read while the last k-step multiplies.
template <int BM, int BN, bool A_KC, bool B_KC, bool VEC>
__global__ __launch_bounds__(kThreads, BM * BN >= 128 * 64 ? 1 : 2)
void gemm_f32_pipe_kernel(GemmParams p) {
  constexpr int BKT = 32;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int KL = BKT / 4;  // k-steps per K-tile (each lane group owns KL consecutive k)
  using SA = Stage<BM, BKT, A_KC, VEC, kThreads>;
  using SB = Stage<BN, BKT, B_KC, VEC, kThreads>;
  constexpr int NS = SA::NV + SB::NV;  // staged float4 per thread per K-tile
  static_assert(NS <= KL - 1, "staging must finish before the barrier step");
  __shared__ __attribute__((aligned(16))) float smem[2 * (SA::SIZE + SB::SIZE)];

  const int nwg = p.tiles_m * p.tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / p.tiles_n;
  const int tn = wg - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int split = blockIdx.y;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;
  const bool mn_full = (m0 + BM <= p.M) && (n0 + BN <= p.N);

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int kq = lane >> 4;
  const int l16 = lane & 15;
  const int wm0 = (wave >> 1) * WM;
  const int wn0 = (wave & 1) * WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = (kend - kbeg + BKT - 1) / BKT;
  SA sa;
  SB sb;
  (void)mn_full;
  // buffer descriptors over exactly the addressed extent (host guarantees < 2 GiB)
  const int64_t a_ext = A_KC ? (p.M - 1) * p.lda + p.K : (p.K - 1) * p.lda + p.M;
  const int64_t b_ext = B_KC ? (p.N - 1) * p.ldb + p.K : (p.K - 1) * p.ldb + p.N;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)(a_ext * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)(b_ext * 4), 0x00020000);
  auto fetch_one = [&](int c, int64_t t) {  // staged float4 c of K-tile t (zeros past nk)
    const int64_t k0 = kbeg + t * BKT;
    if (c < SA::NV)
      sa.load_one4(c, ra, p.lda, m0, p.M, k0, kend, tid);
    else
      sb.load_one4(c - SA::NV, rb, p.ldb, n0, p.N, k0, kend, tid);
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
  auto iteration = [&](int64_t kt, float (&ca)[FM][KL], float (&cb)[FN][KL], float (&na)[FM][KL],
                       float (&nb)[FN][KL]) {
    float* nbuf = smem + ((kt + 1) & 1) * (SA::SIZE + SB::SIZE);
#pragma unroll
    for (int s = 0; s < KL - 1; ++s) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[i][s], cb[j][s], acc[i][j], 0, 0, 0);
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
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[i][KL - 1], cb[j][KL - 1], acc[i][j], 0, 0, 0);
  };
  float a1[FM][KL], b1[FN][KL];
  for (int64_t kt = 0; kt < nk; kt += 2) {
    iteration(kt, a, b, a1, b1);
    if (kt + 1 >= nk) break;
    iteration(kt + 1, a1, b1, a, b);
  }

  // Epilogue: register r of a 16x16 accumulator holds row 4*(lane>>4) + r, col lane&15.
  const bool partial = gridDim.y > 1;
  float* wsp = partial ? p.ws + (int64_t)split * p.M * p.N : nullptr;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = n0 + wn0 + j * 16 + l16;
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm0 + i * 16 + 4 * kq + r;
        if (row >= p.M) continue;
        if (partial)
          wsp[row * p.N + col] = acc[i][j][r];
        else
          apply_epilogue(p, row, col, p.alpha * acc[i][j][r]);
      }
    }
  }
}

// Sum the split partials in split order, scale, apply the epilogue.
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(GemmParams p, int splits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MN = p.M * p.N;
  if (i >= MN) return;
  float s = p.ws[i];
  for (int k = 1; k < splits; ++k) s += p.ws[(int64_t)k * MN + i];
  const int64_t row = i / p.N;
  apply_epilogue(p, row, i - row * p.N, p.alpha * s);
}

struct Plan {
  int bm, bn, bk, splits;
  int64_t kchunk;
  int ks = 1;
};

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

Plan finish_plan(int bm, int bn, int bk, int64_t s, int64_t K) {
  int64_t smax = K / kMinSplitK;
  if (s > smax) s = smax;
  if (s > kMaxSplit) s = kMaxSplit;
  if (s < 1) s = 1;
  int64_t kchunk = dlrm::ceil_div(dlrm::ceil_div(K, s), bk) * bk;
  if (kchunk < bk) kchunk = bk;
  s = dlrm::ceil_div(K, kchunk);
  if (s < 1) s = 1;
  return {bm, bn, bk, (int)s, kchunk};
}

bool valid_cfg(int bm, int bn, int bk, int ks) {
  const bool tile = (bm == 64 || bm == 128) && (bn == 64 || bn == 128);
  if (ks == 16) return tile && bk == 32;
  if (ks == 32) return tile && bk == 32 && bm * bn <= 128 * 64;
  if (ks == 2) return tile && bk == 32 || (bm == 64 && bn == 64 && bk == 64);
  return ks == 1 && tile && (bk == 32 || bk == 64);
}

struct PlanEntry {
  int64_t M, N, K;
  int ta, tb, bm, bn, bk, split, ks;
};

// Measured plans for the DLRM step shapes (exact match), from tools/gemm_sweep.py.
constexpr PlanEntry kPlans[] = {
#include "gemm_plans.inc"
};

// Tuning overrides (read per call, for sweeps): DLRM_GEMM_CFG=<BM>x<BN>x<BK>,
// DLRM_GEMM_SPLIT=<n>, DLRM_GEMM_TARGET=<workgroups>.
Plan plan_gemm(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc) {
  const int force_split = env_int("DLRM_GEMM_SPLIT", 0);
  const char* cfg = getenv("DLRM_GEMM_CFG");
  if (cfg && *cfg) {
    int bm = 64, bn = 64, bk = 32, ks = 1;
    const int n = sscanf(cfg, "%dx%dx%dx%d", &bm, &bn, &bk, &ks);
    if (n < 3) bm = bn = 64, bk = 32;
    if (n < 4) ks = 1;
    if (!valid_cfg(bm, bn, bk, ks)) bm = bn = 64, bk = 32, ks = 1;
    const int64_t s = force_split > 0 ? force_split : 1;
    Plan pl = finish_plan(bm, bn, bk, s, K);
    pl.ks = ks;
    return pl;
  }
  const int ta = a_kc ? 0 : 1, tb = b_kc ? 1 : 0;
  for (const PlanEntry& e : kPlans)
    if (e.M == M && e.N == N && e.K == K && e.ta == ta && e.tb == tb && !getenv("DLRM_GEMM_NOTABLE"))
    {
      Plan pl = finish_plan(e.bm, e.bn, e.bk, e.split, K);
      pl.ks = e.ks;
      return pl;
    }
  // Heuristic: the largest tile that still gives >= target workgroups; split K of the
  // 64x64 tiling up to the target otherwise.
  const int target = env_int("DLRM_GEMM_TARGET", (a_kc && b_kc) ? 512 : 1536);
  const int64_t t128 = dlrm::ceil_div(M, 128) * dlrm::ceil_div(N, 128);
  if (t128 >= target) return {128, 128, 32, 1, K};
  const int64_t t64x128 = dlrm::ceil_div(M, 64) * dlrm::ceil_div(N, 128);
  if (t64x128 >= target) return {64, 128, 32, 1, K};
  const int64_t t64 = dlrm::ceil_div(M, 64) * dlrm::ceil_div(N, 64);
  const int64_t s = force_split > 0 ? force_split : dlrm::ceil_div(target, t64);
  return finish_plan(64, 64, 32, s, K);
}

template <int BM, int BN, int BKT, int KS>
int launch_cfg(GemmParams p, int splits, bool a_kc, bool b_kc, bool vec, hipStream_t st) {
  p.tiles_m = (int)dlrm::ceil_div(p.M, BM);
  p.tiles_n = (int)dlrm::ceil_div(p.N, BN);
  constexpr bool M16 = KS == 16;   // KS == 16 selects the 16x16x4 kernel
  constexpr bool PIPE = KS == 32;  // KS == 32 selects the pipelined 16x16x4 kernel
  const dim3 grid(p.tiles_m * p.tiles_n, splits), block((M16 || PIPE) ? kThreads : kThreads * KS);
#define G(AK, BK_, V_)                                                                          \
  do {                                                                                          \
    if constexpr (PIPE)                                                                         \
      hipLaunchKernelGGL((gemm_f32_pipe_kernel<BM, BN, AK, BK_, V_>), grid, block, 0, st, p);   \
    else if constexpr (M16)                                                                     \
      hipLaunchKernelGGL((gemm_f32_mfma16_kernel<BM, BN, AK, BK_, V_>), grid, block, 0, st, p); \
    else                                                                                        \
      hipLaunchKernelGGL((gemm_f32_mfma_kernel<BM, BN, BKT, ((M16 || PIPE) ? 1 : KS), AK, BK_, V_>), grid, \
                         block, 0, st, p);                                                      \
  } while (0)
#define G_V(AK, BK_)  \
  if (vec)            \
    G(AK, BK_, true); \
  else                \
    G(AK, BK_, false);
  if (a_kc && b_kc) {
    G_V(true, true)
  } else if (a_kc) {
    G_V(true, false)
  } else if (b_kc) {
    G_V(false, true)
  } else {
    G_V(false, false)
  }
#undef G_V
#undef G
  DLRM_LAUNCH_CHECK("dlrm_gemm_f32");
  if (splits > 1) {
    hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(dlrm::ceil_div(p.M * p.N, 256)), dim3(256),
                       0, st, p, splits);
    DLRM_LAUNCH_CHECK("dlrm_gemm_f32 (split-K reduce)");
  }
  return DLRM_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline bool kbeg_ok(int64_t kchunk) { return kchunk % 4 == 0; }

}  // namespace

extern "C" size_t dlrm_gemm_f32_workspace_size(int32_t trans_a, int32_t trans_b, int64_t M,
                                               int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const Plan pl = plan_gemm(M, N, K, !trans_a, trans_b != 0);
  return pl.splits > 1 ? (size_t)pl.splits * M * N * sizeof(float) : 0;
}

extern "C" int dlrm_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K,
                             float alpha, const float* A, int64_t lda, const float* B,
                             int64_t ldb, float* C, int64_t ldc, int32_t epilogue,
                             const float* bias, const float* aux, int64_t ld_aux,
                             void* workspace, size_t workspace_bytes, dlrm_stream_t stream) {
  DLRM_ARG(M >= 0 && N >= 0 && K >= 0, "dlrm_gemm_f32: negative size");
  if (M == 0 || N == 0) return DLRM_OK;
  DLRM_ARG(C, "dlrm_gemm_f32: null C");
  DLRM_ARG(K == 0 || (A && B), "dlrm_gemm_f32: null A/B");
  DLRM_ARG(epilogue >= DLRM_EPI_STORE && epilogue <= DLRM_EPI_RELU, "dlrm_gemm_f32: bad epilogue");
  DLRM_ARG(!(epilogue == DLRM_EPI_BIAS || epilogue == DLRM_EPI_BIAS_RELU) || bias,
           "dlrm_gemm_f32: epilogue needs bias");
  DLRM_ARG(epilogue != DLRM_EPI_DRELU || (aux && ld_aux >= N), "dlrm_gemm_f32: DRELU needs aux");
  DLRM_ARG(ldc >= N, "dlrm_gemm_f32: ldc < N");
  DLRM_ARG(trans_a ? lda >= M : lda >= K, "dlrm_gemm_f32: bad lda");
  DLRM_ARG(trans_b ? ldb >= K : ldb >= N, "dlrm_gemm_f32: bad ldb");
  const int64_t tiles_max = dlrm::ceil_div(M, 64) * dlrm::ceil_div(N, 64);
  DLRM_REQUIRE(tiles_max < (int64_t)INT32_MAX, DLRM_ERR_UNSUPPORTED, "dlrm_gemm_f32: too large");

  GemmParams p{};
  p.M = M;
  p.N = N;
  p.K = K;
  p.alpha = alpha;
  p.A = A;
  p.lda = lda;
  p.B = B;
  p.ldb = ldb;
  p.C = C;
  p.ldc = ldc;
  p.epi = epilogue;
  p.bias = bias;
  p.aux = aux;
  p.ldaux = ld_aux;
  Plan pl = plan_gemm(M, N, K, !trans_a, trans_b != 0);
  if (pl.splits > 1) {
    const size_t need = (size_t)pl.splits * M * N * sizeof(float);
    if (!workspace || workspace_bytes < need) {  // no workspace: single pass
      pl.splits = 1;
      pl.kchunk = K;
    } else {
      p.ws = static_cast<float*>(workspace);
    }
  }
  p.kchunk = pl.kchunk > 0 ? pl.kchunk : 1;
  const bool a_kc = !trans_a;
  const bool b_kc = trans_b != 0;
  const bool vec = aligned16(A) && (lda % 4 == 0) && aligned16(B) && (ldb % 4 == 0);
  // the pipelined kernel moves whole float4s: K and the mn extent of an mn-contiguous
  // operand must be multiples of 4 (else the planner's pick falls back to the 16x16 kernel)
  const int64_t a_ext = a_kc ? (M - 1) * lda + K : (K - 1) * lda + M;
  const int64_t b_ext = b_kc ? (N - 1) * ldb + K : (K - 1) * ldb + N;
  const bool vec4 = vec && K % 4 == 0 && (a_kc || M % 4 == 0) && (b_kc || N % 4 == 0) &&
                    kbeg_ok(pl.kchunk) && a_ext * 4 < 0x7ff00000LL && b_ext * 4 < 0x7ff00000LL;
  if (pl.ks == 32 && !vec4) pl.ks = 16;
  hipStream_t st = dlrm::as_stream(stream);
#define CFG(BM_, BN_, BK_, KS_)                                      \
  if (pl.bm == BM_ && pl.bn == BN_ && pl.bk == BK_ && pl.ks == KS_) \
    return launch_cfg<BM_, BN_, BK_, KS_>(p, pl.splits, a_kc, b_kc, vec, st);
  CFG(64, 64, 32, 1)
  CFG(128, 64, 32, 1)
  CFG(64, 128, 32, 1)
  CFG(128, 128, 32, 1)
  CFG(64, 64, 64, 1)
  CFG(128, 64, 64, 1)
  CFG(64, 128, 64, 1)
  CFG(128, 128, 64, 1)
  CFG(64, 64, 32, 2)
  CFG(128, 64, 32, 2)
  CFG(64, 128, 32, 2)
  CFG(128, 128, 32, 2)
  CFG(64, 64, 64, 2)
  CFG(64, 64, 32, 16)
  CFG(128, 64, 32, 16)
  CFG(64, 128, 32, 16)
  CFG(128, 128, 32, 16)
  CFG(64, 64, 32, 32)
  CFG(128, 64, 32, 32)
  CFG(64, 128, 32, 32)
#undef CFG
  dlrm::set_error("dlrm_gemm_f32: no kernel for plan %dx%dx%dx%d", pl.bm, pl.bn, pl.bk, pl.ks);
  return DLRM_ERR_UNSUPPORTED;
}
