// GEMM body experiments (not product code): tools/gemm_lab.py builds this into
// tools/_lab/libgemm_lab.so and times the library's pipe_body at other tiles, wave layouts,
// occupancies and LDS-stage depths (U 32-deep sub-tiles per barrier) against the library's
// own launch on the C3 step shapes.  Includes the library's gemm.hip, so the body, staging,
// epilogue / split-K completion and planner are the product's own; every result is
// bitwise the library's at the same split (the MFMA order does not depend on the tile or U).
// (Round 5's candidate bodies - fragment groups, LDS-DMA rings - measured slower and left
// with their commit, e02bb7a.)
#ifdef LAB_TRACE
// Timeline build (tools/gemm_trace.py): thread 0 of every workgroup stamps the shader clock
// (s_memtime) at the body's hooks into g_stamps[blockIdx.x][slot]; slot 0 = start, 1 = after
// the prologue, 2 + t = after K-tile t (t < 66), 68 = before the epilogue, 69 = end; 70 / 71 =
// s_memrealtime (100 MHz, chip-wide) at start / end.
#include <hip/hip_runtime.h>
__device__ long long* g_stamps;
#define DLRM_GEMM_STAMP(slot)                                                          \
  do {                                                                                 \
    if (threadIdx.x == 0 && g_stamps) {                                                \
      const int s_ = (slot) < 0 ? 70 + (slot) : ((slot) < 68 ? (slot) : -1);           \
      long long* r_ = g_stamps + (long long)blockIdx.x * 72;                           \
      if (s_ >= 0) r_[s_] = (long long)__builtin_amdgcn_s_memtime();                   \
      if ((slot) == 0) r_[70] = (long long)__builtin_amdgcn_s_memrealtime();           \
      if ((slot) == -1) r_[71] = (long long)__builtin_amdgcn_s_memrealtime();          \
    }                                                                                  \
  } while (0)
extern "C" int lab_set_stamps(void* p) {
  long long* q = static_cast<long long*>(p);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &q, sizeof(q)) == hipSuccess ? 0 : -1;
}
#endif
#include "../dlrm-yx_amd/csrc/gemm.hip"

namespace {

template <int BM, int BN, int WGM, int WGN, int OCC, int KINDS, int U>
__global__ __launch_bounds__(WGM * WGN * 64, OCC) void old_kernel(const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN, U>()];
  // persistent form (grid < g.total): each workgroup walks the virtual blocks b, b + grid, ...
  for (int b = blockIdx.x; b < g.total; b += gridDim.x) {
    group_body<BM, BN, WGM, WGN, KINDS, U>(g, b, smem);
    __syncthreads();  // the next tile's prologue rewrites the LDS images
  }
}

template <int BM, int BN, int WGM, int WGN>
int lab_prepare(int n, const Desc* d, const Plan* pl, void* ws, size_t ws_bytes, GemmGroup& g) {
  constexpr int NT = WGM * WGN * 64;
  g = GemmGroup{};
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
  if (tick > kTicketCap || (tick && ws_bytes < c.used)) return -1;
  g.total = (int)blocks;
  return 0;
}

// Workgroups per CU capped at g_cap (> 0) by a dynamic-LDS pad: the dispatcher then cannot
// pack more than g_cap of this launch's workgroups onto one CU (tests whether uneven packing
// of the 2-6 that fit by registers / LDS is what the per-CU rate loses).
int g_cap = 0;
int g_persist = 0;  // > 0: grid = min(total, g_persist * 256) workgroups looping over the tiles
template <int BM, int BN, int WGM, int WGN, int OCC, int U, int KINDS>
void lab_go(const GemmGroup& g, hipStream_t st) {
  const int nwg = g_persist > 0 && g.total > g_persist * 256 ? g_persist * 256 : g.total;
  const dim3 grid(nwg), block(WGM * WGN * 64);
  size_t pad = 0;
  if (g_cap > 0) {
    const size_t stat = group_smem_floats<BM, BN, U>() * sizeof(float);
    const size_t per = 163840 / g_cap - 1024;
    pad = per > stat ? per - stat : 0;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&old_kernel<BM, BN, WGM, WGN, OCC, KINDS, U>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
  }
  hipLaunchKernelGGL((old_kernel<BM, BN, WGM, WGN, OCC, KINDS, U>), grid, block, pad, st, g);
}

template <int BM, int BN, int WGM, int WGN, int OCC, int U>
int lab_launch(int n, const Desc* d, const Plan* pl, void* ws, size_t ws_bytes, hipStream_t st) {
  GemmGroup g;
  if (lab_prepare<BM, BN, WGM, WGN>(n, d, pl, ws, ws_bytes, g)) return -1;
  int kinds = 0;
  for (int i = 0; i < n; ++i)
    if (g.p[i].mode != DLRM_GEMM_REDUCE)
      kinds |= kind_bit(g.p[i].layout, g.p[i].layout == 2 && g.p[i].ones_col >= 0);
  switch (kinds) {
    case 1: lab_go<BM, BN, WGM, WGN, OCC, U, 1>(g, st); break;
    case 2: lab_go<BM, BN, WGM, WGN, OCC, U, 2>(g, st); break;
    case 4: lab_go<BM, BN, WGM, WGN, OCC, U, 4>(g, st); break;
    case 16: lab_go<BM, BN, WGM, WGN, OCC, U, 16>(g, st); break;
    default: lab_go<BM, BN, WGM, WGN, OCC, U, 31>(g, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace

extern "C" int lab_gemm(int32_t cfg, int32_t split, int32_t n, const dlrm_gemm_problem* probs,
                        void* ws, size_t ws_bytes, dlrm_stream_t stream) {
  Desc d[kMaxGroup];
  Plan pl[kMaxGroup];
  for (int i = 0; i < n; ++i) {
    d[i] = desc_of(probs[i]);
    if (d[i].mode == DLRM_GEMM_PARTIAL) pl[i] = make_plan(d[i].splits, d[i].K);
    else pl[i] = make_plan(split > 0 ? split : 1, d[i].K);
  }
  hipStream_t st = dlrm::as_stream(stream);
  // cfg = persist * 10000 + cap * 1000 + U * 100 + tile: at most `cap` workgroups per CU;
  // persist > 0: persist * 256 workgroups, each looping over tiles (b, b + grid, ...)
  g_persist = cfg / 10000;
  g_cap = (cfg / 1000) % 10;
  cfg %= 1000;
  // cfg = U * 100 + tile: tile 0: 64x32, 1: 64x64, 2: 128x64, 3: 64x128, 4: 32x32,
  // 5: 128x64 on 4x2 waves, 6: 128x128 on 4x2 waves, 7: 64x64 at one workgroup per CU
  switch (cfg) {
#define C_(U_)                                                                              \
  case U_ * 100 + 0: return lab_launch<64, 32, 2, 2, 2, U_>(n, d, pl, ws, ws_bytes, st);    \
  case U_ * 100 + 1: return lab_launch<64, 64, 2, 2, 2, U_>(n, d, pl, ws, ws_bytes, st);    \
  case U_ * 100 + 2: return lab_launch<128, 64, 2, 2, 1, U_>(n, d, pl, ws, ws_bytes, st);   \
  case U_ * 100 + 3: return lab_launch<64, 128, 2, 2, 1, U_>(n, d, pl, ws, ws_bytes, st);   \
  case U_ * 100 + 4: return lab_launch<32, 32, 2, 2, 4, U_>(n, d, pl, ws, ws_bytes, st);    \
  case U_ * 100 + 5: return lab_launch<128, 64, 4, 2, 1, U_>(n, d, pl, ws, ws_bytes, st);   \
  case U_ * 100 + 7: return lab_launch<64, 64, 2, 2, 1, U_>(n, d, pl, ws, ws_bytes, st);
    C_(1) C_(2)
#undef C_
    case 106: return lab_launch<128, 128, 4, 2, 1, 1>(n, d, pl, ws, ws_bytes, st);
    case 206: return lab_launch<128, 128, 4, 2, 1, 2>(n, d, pl, ws, ws_bytes, st);
    case 400: return lab_launch<64, 32, 2, 2, 1, 4>(n, d, pl, ws, ws_bytes, st);
    case 401: return lab_launch<64, 64, 2, 2, 1, 4>(n, d, pl, ws, ws_bytes, st);
    case 404: return lab_launch<32, 32, 2, 2, 2, 4>(n, d, pl, ws, ws_bytes, st);
    default: return -3;
  }
}
