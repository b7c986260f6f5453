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
template <int MN, int BKT, bool KC, bool VEC>
struct Stage {
  static constexpr int PITCH = KC ? BKT + 4 : MN + 4;
  static constexpr int SIZE = KC ? MN * PITCH : BKT * PITCH;  // floats per LDS buffer
  static constexpr int NV = MN * BKT / 4 / kThreads;         // float4 per thread
  static_assert(NV >= 1 && MN * BKT % (4 * kThreads) == 0, "panel / thread mismatch");
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
        coords(tid + v * kThreads, mn, k);
        const float* ptr = KC ? X + (mn0 + mn) * ld + k0 + k : X + (k0 + k) * ld + mn0 + mn;
        regs[v] = *reinterpret_cast<const float4*>(ptr);
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int mn, k;
      coords(tid + v * kThreads, mn, k);
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

  __device__ __forceinline__ void store(float* __restrict__ lds, int tid) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int mn, k;
      coords(tid + v * kThreads, mn, k);
      float* dst = KC ? lds + mn * PITCH + k : lds + k * PITCH + mn;
      *reinterpret_cast<float4*>(dst) = regs[v];
    }
  }

  // 16 consecutive k-steps (k = kbase .. kbase+15) of the 32-wide sub-tile at `off`
  // for this lane (row/col off + l32).
  __device__ __forceinline__ void frag(const float* __restrict__ lds, int off, int l32, int kbase,
                                       float (&f)[16]) const {
    if constexpr (KC) {
      const float* p = lds + (off + l32) * PITCH + kbase;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * c);
        f[4 * c + 0] = v.x;
        f[4 * c + 1] = v.y;
        f[4 * c + 2] = v.z;
        f[4 * c + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) f[s] = lds[(kbase + s) * PITCH + off + l32];
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

template <int BM, int BN, int BKT, bool A_KC, bool B_KC, bool VEC>
__global__ __launch_bounds__(kThreads, (BM * BN >= 128 * 128 && BKT >= 64) ? 1 : 2)
void gemm_f32_mfma_kernel(GemmParams p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  using SA = Stage<BM, BKT, A_KC, VEC>;
  using SB = Stage<BN, BKT, B_KC, VEC>;
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
    for (int sub = 0; sub < BKT / 32; ++sub) {
      const int kbase = h * (BKT / 2) + sub * 16;
      float a[TM][16], b[TN][16];
#pragma unroll
      for (int i = 0; i < TM; ++i) sa.frag(As, wm0 + i * 32, l32, kbase, a[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) sb.frag(Bs, wn0 + j * 32, l32, kbase, b[j]);
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(odd ? As0 : As1, tid);
      sb.store(odd ? Bs0 : Bs1, tid);
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
  int bm, bn, bk, splits;
  int64_t kchunk;
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

bool valid_cfg(int bm, int bn, int bk) {
  const bool tile = (bm == 64 || bm == 128) && (bn == 64 || bn == 128);
  return tile && (bk == 32 || bk == 64);
}

struct PlanEntry {
  int64_t M, N, K;
  int ta, tb, bm, bn, bk, split;
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
    int bm = 64, bn = 64, bk = 32;
    if (sscanf(cfg, "%dx%dx%d", &bm, &bn, &bk) != 3 || !valid_cfg(bm, bn, bk)) bm = bn = 64, bk = 32;
    const int64_t t = dlrm::ceil_div(M, bm) * dlrm::ceil_div(N, bn);
    const int64_t s = force_split > 0 ? force_split : 1;
    (void)t;
    return finish_plan(bm, bn, bk, s, K);
  }
  const int ta = a_kc ? 0 : 1, tb = b_kc ? 1 : 0;
  for (const PlanEntry& e : kPlans)
    if (e.M == M && e.N == N && e.K == K && e.ta == ta && e.tb == tb && !getenv("DLRM_GEMM_NOTABLE"))
      return finish_plan(e.bm, e.bn, e.bk, e.split, K);
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

template <int BM, int BN, int BKT>
int launch_cfg(GemmParams p, int splits, bool a_kc, bool b_kc, bool vec, hipStream_t st) {
  p.tiles_m = (int)dlrm::ceil_div(p.M, BM);
  p.tiles_n = (int)dlrm::ceil_div(p.N, BN);
  const dim3 grid(p.tiles_m * p.tiles_n, splits), block(kThreads);
#define G(AK, BK_, V_) \
  hipLaunchKernelGGL((gemm_f32_mfma_kernel<BM, BN, BKT, AK, BK_, V_>), grid, block, 0, st, p)
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
  hipStream_t st = dlrm::as_stream(stream);
#define CFG(BM_, BN_, BK_)                       \
  if (pl.bm == BM_ && pl.bn == BN_ && pl.bk == BK_) \
    return launch_cfg<BM_, BN_, BK_>(p, pl.splits, a_kc, b_kc, vec, st);
  CFG(64, 64, 32)
  CFG(128, 64, 32)
  CFG(64, 128, 32)
  CFG(128, 128, 32)
  CFG(64, 64, 64)
  CFG(128, 64, 64)
  CFG(64, 128, 64)
  CFG(128, 128, 64)
#undef CFG
  dlrm::set_error("dlrm_gemm_f32: no kernel for plan %dx%dx%d", pl.bm, pl.bn, pl.bk);
  return DLRM_ERR_UNSUPPORTED;
}
