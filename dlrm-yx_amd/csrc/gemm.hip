// Exact-fp32 GEMM with fused epilogues on the gfx950 fp32 matrix core
// (v_mfma_f32_32x32x2_f32: 64 FLOP/clk/SIMD, bit-exact k-ordered fmaf chain, no xf32).
//
// Serves the DLRM MLPs (DLRM_Net.create_mlp / apply_mlp, dlrm_s_pytorch.py:227-265,
// 518-524): Linear forward with bias(+ReLU) fused, dgrad with the ReLU mask of the
// previous activation fused, wgrad with the SGD update fused (single GPU) or stored
// into the flat gradient bucket (multi GPU, all-reduced before the update).
//
// Structure: 256-thread workgroups = 4 waves in a 2x2 arrangement, each wave owning a
// (BM/2)x(BN/2) sub-tile built from 32x32 MFMA accumulators (16 AGPRs each).  K is
// staged BK=32 deep through double-buffered LDS in k-major rows ([k][m], [k][n]) so
// each MFMA operand fetch is one conflict-free ds_read_b32 per lane (32 consecutive
// floats per half-wave).  Operands that are k-contiguous in HBM (X rows, W rows of
// nn.Linear) are transposed on the LDS write with an odd row pitch (conflict-free
// ds_write_b32); mn-contiguous operands go in with ds_write_b128.  The next K-tile is
// fetched into registers before the MFMAs of the current one (global latency hidden
// under 64-cycle MFMAs) and written after them, one barrier per K-tile.  Workgroups
// are remapped bijectively so that each XCD (private 4 MiB L2) receives a contiguous
// run of output tiles that share operand panels.
//
// DLRM's GEMMs are small for 256 CUs (M = batch <= 2048, N,K <= 1024) and the weight
// gradients have a long K (= the batch) over a small M x N: the planner splits K
// until there are >= 2 workgroups per CU; split partials go to a caller workspace and
// a reduce kernel sums them IN SPLIT ORDER (deterministic) and applies the epilogue.
#include <cstdlib>

#include "common.hpp"

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int BK = 32;
constexpr int kTargetWG = 512;  // 2 workgroups per CU
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

// Stages an (MN x BK) panel of X into LDS rows [BK][MN + PAD].
//   KCONTIG: X(mn, k) = X[mn*ld + k]     (float4 along k, transposed on the LDS write)
//   else   : X(mn, k) = X[k*ld + mn]     (float4 along mn, direct ds_write_b128)
template <int MN, bool KCONTIG, bool VEC>
struct TileLoader {
  static constexpr int NV = MN * BK / 4 / 256;  // float4 per thread
  static constexpr int PAD = KCONTIG ? 1 : 4;
  static constexpr int STRIDE = MN + PAD;
  static constexpr int SIZE = BK * STRIDE;  // floats per LDS stage
  float4 regs[NV];

  __device__ __forceinline__ void load(const float* __restrict__ X, int64_t ld, int64_t mn0,
                                       int64_t mnlim, int64_t k0, int64_t klim, int tid) {
    // Workgroup-uniform fast path: the whole panel is in range -> plain float4 loads.
    if (VEC && mn0 + MN <= mnlim && k0 + BK <= klim) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int q = tid + v * 256;
        const float* ptr;
        if constexpr (KCONTIG)
          ptr = X + (mn0 + q / (BK / 4)) * ld + k0 + 4 * (q % (BK / 4));
        else
          ptr = X + (k0 + q / (MN / 4)) * ld + mn0 + 4 * (q % (MN / 4));
        regs[v] = *reinterpret_cast<const float4*>(ptr);
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int q = tid + v * 256;
      int64_t gmn, gk;
      if constexpr (KCONTIG) {
        gmn = mn0 + q / (BK / 4);
        gk = k0 + 4 * (q % (BK / 4));
      } else {
        gk = k0 + q / (MN / 4);
        gmn = mn0 + 4 * (q % (MN / 4));
      }
      float e[4];
      bool full;
      const float* ptr;
      if constexpr (KCONTIG) {
        full = (gmn < mnlim) && (gk + 3 < klim);
        ptr = X + gmn * ld + gk;
      } else {
        full = (gk < klim) && (gmn + 3 < mnlim);
        ptr = X + gk * ld + gmn;
      }
      if (VEC && full) {
        regs[v] = *reinterpret_cast<const float4*>(ptr);
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          bool ok;
          if constexpr (KCONTIG)
            ok = (gmn < mnlim) && (gk + c < klim);
          else
            ok = (gk < klim) && (gmn + c < mnlim);
          e[c] = ok ? ptr[c] : 0.f;
        }
        regs[v] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ lds, int tid) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int q = tid + v * 256;
      if constexpr (KCONTIG) {
        const int mn = q / (BK / 4);
        const int kq = q % (BK / 4);
        lds[(4 * kq + 0) * STRIDE + mn] = regs[v].x;
        lds[(4 * kq + 1) * STRIDE + mn] = regs[v].y;
        lds[(4 * kq + 2) * STRIDE + mn] = regs[v].z;
        lds[(4 * kq + 3) * STRIDE + mn] = regs[v].w;
      } else {
        const int k = q / (MN / 4);
        const int mq = q % (MN / 4);
        *reinterpret_cast<float4*>(lds + k * STRIDE + 4 * mq) = regs[v];
      }
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

template <int BM, int BN, bool A_KC, bool B_KC, bool VA, bool VB>
__global__ __launch_bounds__(256, 2) void gemm_f32_mfma_kernel(GemmParams p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  using LA = TileLoader<BM, A_KC, VA>;
  using LB = TileLoader<BN, B_KC, VB>;
  __shared__ __attribute__((aligned(16))) float smem[2 * (LA::SIZE + LB::SIZE)];
  float* As0 = smem;
  float* Bs0 = smem + LA::SIZE;
  float* As1 = smem + LA::SIZE + LB::SIZE;
  float* Bs1 = As1 + LA::SIZE;

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
  const int h = lane >> 5;
  const int l32 = lane & 31;
  const int wm0 = (wave >> 1) * WM;
  const int wn0 = (wave & 1) * WN;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  LA la;
  LB lb;
  const int64_t nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    la.load(p.A, p.lda, m0, p.M, kbeg, kend, tid);
    lb.load(p.B, p.ldb, n0, p.N, kbeg, kend, tid);
    la.store(As0, tid);
    lb.store(Bs0, tid);
  }
  __syncthreads();

  for (int64_t kt = 0; kt < nk; ++kt) {
    const bool odd = kt & 1;
    const float* As = odd ? As1 : As0;
    const float* Bs = odd ? Bs1 : Bs0;
    const bool more = kt + 1 < nk;
    if (more) {
      la.load(p.A, p.lda, m0, p.M, kbeg + (kt + 1) * BK, kend, tid);
      lb.load(p.B, p.ldb, n0, p.N, kbeg + (kt + 1) * BK, kend, tid);
    }
    // All operands of the K-tile are fetched into registers first (the LDS reads are
    // independent, so they stay in flight under the MFMA chain instead of exposing
    // their latency once per k-step), then the MFMAs consume them.
    float a[BK / 2][TM], b[BK / 2][TN];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) a[s][i] = As[(2 * s + h) * LA::STRIDE + wm0 + i * 32 + l32];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[s][j] = Bs[(2 * s + h) * LB::STRIDE + wn0 + j * 32 + l32];
    }
#pragma unroll
    for (int s = 0; s < BK / 2; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][i], b[s][j], acc[i][j], 0, 0, 0);
    if (more) {
      la.store(odd ? As0 : As1, tid);
      lb.store(odd ? Bs0 : Bs1, tid);
    }
    __syncthreads();
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
  int bm, bn, splits;
  int64_t kchunk;
};

// Tuning overrides (read per call, for sweeps): DLRM_GEMM_TILE=128x128|128x64|64x128|64x64,
// DLRM_GEMM_SPLIT=<n>, DLRM_GEMM_TARGET=<workgroups>.
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

Plan finish_plan(int bm, int bn, int64_t s, int64_t K) {
  int64_t smax = K / kMinSplitK;
  if (s > smax) s = smax;
  if (s > kMaxSplit) s = kMaxSplit;
  if (s < 1) s = 1;
  int64_t kchunk = dlrm::ceil_div(dlrm::ceil_div(K, s), BK) * BK;
  if (kchunk < BK) kchunk = BK;
  s = dlrm::ceil_div(K, kchunk);
  if (s < 1) s = 1;
  return {bm, bn, (int)s, kchunk};
}

// Workgroup target: measured on MI355X over the C3 step shapes (tools/gemm_sweep.py) —
// forward (X W^T, both operands k-contiguous) peaks at ~2 WGs/CU with no split, the
// dgrad / wgrad forms (one mn-contiguous operand) keep gaining up to ~6 WGs/CU.
Plan plan_gemm(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc) {
  const int target = env_int("DLRM_GEMM_TARGET", (a_kc && b_kc) ? kTargetWG : 3 * kTargetWG);
  const int force_split = env_int("DLRM_GEMM_SPLIT", 0);
  const char* tile = getenv("DLRM_GEMM_TILE");
  if (tile && *tile) {
    int bm = 64, bn = 64;
    if (sscanf(tile, "%dx%d", &bm, &bn) != 2) bm = bn = 64;
    const int64_t t = dlrm::ceil_div(M, bm) * dlrm::ceil_div(N, bn);
    const int64_t s = force_split > 0 ? force_split : dlrm::ceil_div(target, t);
    return finish_plan(bm, bn, s, K);
  }
  const int64_t t128 = dlrm::ceil_div(M, 128) * dlrm::ceil_div(N, 128);
  if (t128 >= target) return {128, 128, 1, K};
  const int64_t t64x128 = dlrm::ceil_div(M, 64) * dlrm::ceil_div(N, 128);
  if (t64x128 >= target) return {64, 128, 1, K};
  const int64_t t64 = dlrm::ceil_div(M, 64) * dlrm::ceil_div(N, 64);
  const int64_t s = force_split > 0 ? force_split : dlrm::ceil_div(target, t64);
  return finish_plan(64, 64, s, K);
}

template <int BM, int BN>
int launch_tiles(GemmParams p, int splits, bool a_kc, bool b_kc, bool va, bool vb,
                 hipStream_t st) {
  p.tiles_m = (int)dlrm::ceil_div(p.M, BM);
  p.tiles_n = (int)dlrm::ceil_div(p.N, BN);
  const dim3 grid(p.tiles_m * p.tiles_n, splits), block(256);
#define G(AK, BK_, VA_, VB_) \
  hipLaunchKernelGGL((gemm_f32_mfma_kernel<BM, BN, AK, BK_, VA_, VB_>), grid, block, 0, st, p)
#define G_V(AK, BK_)          \
  if (va && vb)               \
    G(AK, BK_, true, true);   \
  else if (va)                \
    G(AK, BK_, true, false);  \
  else if (vb)                \
    G(AK, BK_, false, true);  \
  else                        \
    G(AK, BK_, false, false);
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
  const bool va = aligned16(A) && (lda % 4 == 0);
  const bool vb = aligned16(B) && (ldb % 4 == 0);
  hipStream_t st = dlrm::as_stream(stream);
  if (pl.bm == 128 && pl.bn == 128)
    return launch_tiles<128, 128>(p, pl.splits, a_kc, b_kc, va, vb, st);
  if (pl.bm == 128) return launch_tiles<128, 64>(p, pl.splits, a_kc, b_kc, va, vb, st);
  if (pl.bn == 128) return launch_tiles<64, 128>(p, pl.splits, a_kc, b_kc, va, vb, st);
  return launch_tiles<64, 64>(p, pl.splits, a_kc, b_kc, va, vb, st);
}
