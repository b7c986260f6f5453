// GEMM body experiments (not product code): tools/gemm_lab.py builds this into
// tools/_lab/libgemm_lab.so and times candidate bodies against the library's pipe_body on
// the C3 step shapes.  Includes the library's gemm.hip so the staging helpers, the
// epilogue / split-K completion and the planner are the product's own.
#include "../dlrm-yx_amd/csrc/gemm.hip"

namespace {

// Candidate body: per-wave FM x FN 16x16x4 tiles, BK = 32, LDS double buffer, ONE barrier
// per K-tile, fragments read in two groups of four k-steps (group 1 of tile t under group
// 0's MFMAs, group 0 of tile t+1 right after the barrier under group 1's MFMAs), the next
// tile's staged registers written to LDS and the tile after it fetched during group 0.
template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, bool RS, int PRIO>
__device__ __forceinline__ void body2(const GemmParams& p, int lb, float* smem) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile");
  using SA = Stage<BM, kBK, A_KC, true, NT>;
  using SB = Stage<BN, kBK, B_KC, true, NT>;
  constexpr int NS = SA::NV + SB::NV;

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
  float rs[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) rs[i] = 0.f;

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
  auto put_one = [&](int c, float* buf) {
    if (c < SA::NV)
      sa.store_one(c, buf, tid);
    else
      sb.store_one(c - SA::NV, buf + SA::SIZE, tid);
  };
  // fragments of k-steps 4g .. 4g+3 (lane quarter kq owns k = kq*8 + 4g + 0..3)
  auto read_grp = [&](const float* buf, int g, float (&a)[FM][4], float (&b)[FN][4]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) sa.template frag<4>(buf, wm0 + i * 16, l16, kq * 8 + 4 * g, a[i]);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      sb.template frag<4>(buf + SA::SIZE, wn0 + j * 16, l16, kq * 8 + 4 * g, b[j]);
  };
  auto mfma_step = [&](const float (&a)[FM][4], const float (&b)[FN][4], int s) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    if constexpr (RS) {
#pragma unroll
      for (int i = 0; i < FM; ++i) rs[i] = add_f32(rs[i], a[i][s]);
    }
  };
  constexpr int SZ = SA::SIZE + SB::SIZE;
  float a0[FM][4], b0[FN][4], a1[FM][4], b1[FN][4];
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 0);
#pragma unroll
  for (int c = 0; c < NS; ++c) put_one(c, smem);
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch_one(c, 1);
  __syncthreads();
  read_grp(smem, 0, a0, b0);
  if constexpr (PRIO) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const float* cur = smem + (kt & 1) * SZ;
    float* nxt = smem + ((kt + 1) & 1) * SZ;
    read_grp(cur, 1, a1, b1);
    // group 0: MFMAs; tile t+1 (staged) -> LDS, then tile t+2 -> the staging registers
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      mfma_step(a0, b0, s);
      constexpr int PER = (NS + 3) / 4;
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int c = s * PER + u;
        if (c < NS) {
          put_one(c, nxt);
          fetch_one(c, kt + 2);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    read_grp(nxt, 0, a0, b0);  // tile t+1 group 0 (unused past the last tile)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s) mfma_step(a1, b1, s);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
  }
  finish_tile<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0, smem);
}

template <int BM, int BN, int WGM, int WGN, int PRIO, int KINDS>
__device__ __forceinline__ void lab_group_body(const GemmGroup& g, int b, float* smem) {
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
    if (kind == 0) return body2<BM, BN, WGM, WGN, true, true, false, PRIO>(p, lb, smem);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return body2<BM, BN, WGM, WGN, true, false, false, PRIO>(p, lb, smem);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return body2<BM, BN, WGM, WGN, false, false, false, PRIO>(p, lb, smem);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return body2<BM, BN, WGM, WGN, false, true, false, PRIO>(p, lb, smem);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return body2<BM, BN, WGM, WGN, false, false, true, PRIO>(p, lb, smem);
}

template <int BM, int BN, int WGM, int WGN, int OCC, int PRIO, int KINDS>
__global__ __launch_bounds__(WGM * WGN * 64, OCC) void lab_kernel(const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN>()];
  lab_group_body<BM, BN, WGM, WGN, PRIO, KINDS>(g, blockIdx.x, smem);
}

// the library's body at other wave layouts (for comparison)
template <int BM, int BN, int WGM, int WGN, int OCC, int KINDS>
__global__ __launch_bounds__(WGM * WGN * 64, OCC) void old_kernel(const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[group_smem_floats<BM, BN>()];
  group_body<BM, BN, WGM, WGN, KINDS>(g, blockIdx.x, smem);
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

template <int BM, int BN, int WGM, int WGN, int OCC, int PRIO, bool OLD, int KINDS>
void lab_go(const GemmGroup& g, hipStream_t st) {
  const dim3 grid(g.total), block(WGM * WGN * 64);
  if constexpr (OLD)
    hipLaunchKernelGGL((old_kernel<BM, BN, WGM, WGN, OCC, KINDS>), grid, block, 0, st, g);
  else
    hipLaunchKernelGGL((lab_kernel<BM, BN, WGM, WGN, OCC, PRIO, KINDS>), grid, block, 0, st, g);
}

template <int BM, int BN, int WGM, int WGN, int OCC, int PRIO, bool OLD>
int lab_launch(int n, const Desc* d, const Plan* pl, void* ws, size_t ws_bytes, hipStream_t st) {
  GemmGroup g;
  if (lab_prepare<BM, BN, WGM, WGN>(n, d, pl, ws, ws_bytes, g)) return -1;
  int kinds = 0;
  for (int i = 0; i < n; ++i)
    if (g.p[i].mode != DLRM_GEMM_REDUCE)
      kinds |= kind_bit(g.p[i].layout, g.p[i].layout == 2 && g.p[i].ones_col >= 0);
  switch (kinds) {
    case 1: lab_go<BM, BN, WGM, WGN, OCC, PRIO, OLD, 1>(g, st); break;
    case 2: lab_go<BM, BN, WGM, WGN, OCC, PRIO, OLD, 2>(g, st); break;
    case 4: lab_go<BM, BN, WGM, WGN, OCC, PRIO, OLD, 4>(g, st); break;
    case 16: lab_go<BM, BN, WGM, WGN, OCC, PRIO, OLD, 16>(g, st); break;
    case 18: lab_go<BM, BN, WGM, WGN, OCC, PRIO, OLD, 18>(g, st); break;
    default: lab_go<BM, BN, WGM, WGN, OCC, PRIO, OLD, 31>(g, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace

// cfg: body * 100 + variant; body 1 = the library's pipe_body, 2 = body2.
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
  switch (cfg) {
    case 100: return lab_launch<64, 32, 2, 2, 2, 0, true>(n, d, pl, ws, ws_bytes, st);
    case 101: return lab_launch<64, 64, 2, 2, 2, 0, true>(n, d, pl, ws, ws_bytes, st);
    case 102: return lab_launch<128, 64, 2, 2, 2, 0, true>(n, d, pl, ws, ws_bytes, st);
    case 103: return lab_launch<128, 128, 4, 2, 1, 0, true>(n, d, pl, ws, ws_bytes, st);
    case 200: return lab_launch<64, 32, 2, 2, 2, 0, false>(n, d, pl, ws, ws_bytes, st);
    case 201: return lab_launch<64, 64, 2, 2, 2, 0, false>(n, d, pl, ws, ws_bytes, st);
    case 202: return lab_launch<128, 64, 2, 2, 2, 0, false>(n, d, pl, ws, ws_bytes, st);
    case 203: return lab_launch<128, 128, 4, 2, 1, 0, false>(n, d, pl, ws, ws_bytes, st);
    case 204: return lab_launch<128, 128, 4, 2, 1, 1, false>(n, d, pl, ws, ws_bytes, st);
    case 205: return lab_launch<128, 64, 4, 2, 1, 0, false>(n, d, pl, ws, ws_bytes, st);
    case 206: return lab_launch<128, 64, 4, 2, 1, 1, false>(n, d, pl, ws, ws_bytes, st);
    case 207: return lab_launch<64, 128, 2, 2, 2, 0, false>(n, d, pl, ws, ws_bytes, st);
    case 208: return lab_launch<128, 128, 2, 2, 1, 0, false>(n, d, pl, ws, ws_bytes, st);
    case 209: return lab_launch<256, 64, 4, 2, 1, 0, false>(n, d, pl, ws, ws_bytes, st);
    default: return -3;
  }
}
