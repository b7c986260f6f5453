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

// ---------------------------------------------------------------------------------------
// Ring body (measured slower than pipe_body in the step shapes: profiles/r05_gemm_ring_lab.txt):
// LDS-DMA staging (global_load_lds_dwordx4: no staging registers), an NB-stage ring
// of unpadded K-tile images (BK = 32) with 16-B chunks XOR-swizzled on the SOURCE address
// (the DMA writes lane-linear), loads issued NB-1 K-tiles ahead, one raw barrier per K-tile.
// Same per-element accumulation order as pipe_body (lane quarter kq owns k = kq*8 + s of each
// K-tile, k-steps s = 0..7 in order), so results are bitwise pipe_body's at the same split.
//   KC  image: [mn][32], chunk c of row r at c ^ swz_kc(r): ds_read_b128 conflict-free
//   !KC image: [32][MN], chunk c of k-row k at c ^ 4*((k >> 3) & 1): ds_read_b32 conflict-free
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// One LDS-DMA piece: 64 lanes x 16 B from per-lane sources to LDS bytes [lds, lds + 1 KiB).
// Inline asm (M0 written in the same statement): hipcc neither counts it nor waits for it -
// the K-tile waits below are the only vmcnt waits of the main loop.
__device__ __forceinline__ void glds16(const float* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)p);
}

template <int MN, bool KC, int NW>
struct GPanel {
  static constexpr int FLOATS = MN * 32;
  static constexpr int CH = MN * 8;
  static constexpr int G = CH / (64 * NW);  // LDS-DMA instructions per wave per K-tile
  static_assert(G >= 1 && CH % (64 * NW) == 0, "panel / wave mismatch");
  const float* src[G];  // this lane's chunk at K-tile 0 (mn clamped into range)
  int kpos[G];          // the chunk's k within a K-tile (KC: 4c, !KC: its k-row)

  __device__ __forceinline__ void init(const float* X, int64_t ld, int64_t mn0, int64_t mnlim,
                                       int64_t kbeg, int wave, int lane) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int j = (g * NW + wave) * 64 + lane;
      int mn, k;
      if constexpr (KC) {
        const int r = j >> 3;
        mn = r;
        k = 4 * ((j & 7) ^ swz_kc(r));
      } else {
        constexpr int PER = MN / 4;
        k = j / PER;
        mn = 4 * ((j % PER) ^ (((k >> 3) & 1) * 4));
      }
      int64_t gmn = mn0 + mn;
      if (gmn >= mnlim) gmn = KC ? mnlim - 1 : mnlim - 4;  // rows/cols past the operand:
      // any in-range data (their products land only in outputs that are never written)
      src[g] = KC ? X + gmn * ld + kbeg + k : X + (kbeg + k) * ld + gmn;
      kpos[g] = k;
    }
  }
  // K-tile t of the split into the stage image at `dst`; chunks past the split's K read the
  // operand's first float4 instead (in range) and are zeroed by fix() once landed.
  __device__ __forceinline__ void issue(const float* X, int64_t ld, int t, int krel, float* dst,
                                        int wave) const {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool ok = t * 32 + kpos[g] < krel;
      const float* s = ok ? src[g] + (KC ? (int64_t)t * 32 : (int64_t)t * 32 * ld) : X;
      glds16(s, lds_addr(dst + (g * NW + wave) * 256));
    }
  }
  __device__ __forceinline__ void fix(int t, int krel, float* dst, int wave, int lane) const {
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (t * 32 + kpos[g] >= krel)
        *reinterpret_cast<float4*>(dst + ((g * NW + wave) * 64 + lane) * 4) =
            make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // the 8 k-values (k = kq*8 + s) of row/column off + l16
  __device__ __forceinline__ void frag(const float* img, int off, int l16, int kq,
                                       float (&f)[8]) const {
    if constexpr (KC) {
      const int sw = swz_kc(l16);
      const float* r = img + (off + l16) * 32;
      const float4 v0 = *reinterpret_cast<const float4*>(r + 4 * ((2 * kq) ^ sw));
      const float4 v1 = *reinterpret_cast<const float4*>(r + 4 * ((2 * kq + 1) ^ sw));
      f[0] = v0.x, f[1] = v0.y, f[2] = v0.z, f[3] = v0.w;
      f[4] = v1.x, f[5] = v1.y, f[6] = v1.z, f[7] = v1.w;
    } else {
      const int col = (off + l16) ^ ((kq & 1) << 4);
#pragma unroll
      for (int s = 0; s < 8; ++s) f[s] = img[(kq * 8 + s) * MN + col];
    }
  }
};

template <int BM, int BN, int NB>
constexpr int ring_smem_floats() {
  return NB * (BM + BN) * 32;
}

template <int BM, int BN, int WGM, int WGN, bool A_KC, bool B_KC, bool RS, int NB>
__device__ __forceinline__ void ring_body(const GemmParams& p, int lb, float* smem) {
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave sub-tile");
  using PA = GPanel<BM, A_KC, NW>;
  using PB = GPanel<BN, B_KC, NW>;
  constexpr int G = PA::G + PB::G;
  constexpr int SZ = PA::FLOATS + PB::FLOATS;
  static_assert(NB >= 2 && G * (NB - 2) < 64, "ring depth");

  const int tile = lb / p.splits;
  const int split = lb - tile * p.splits;
  const int tm = tile / p.tiles_n;
  const int tn = tile - tm * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)split * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;
  const int krel = (int)(kend - kbeg);
  const int nk = (krel + 31) / 32;
  const bool ragged = (krel & 31) != 0;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  PA pa;
  PB pb;
  pa.init(p.A, p.lda, m0, p.M, kbeg, wave, lane);
  pb.init(p.B, p.ldb, n0, p.N, kbeg, wave, lane);
  auto stage = [&](int t) { return smem + (t % NB) * SZ; };
  auto issue = [&](int t) {
    float* st = stage(t);
    pa.issue(p.A, p.lda, t, krel, st, wave);
    pb.issue(p.B, p.ldb, t, krel, st + PA::FLOATS, wave);
  };
  auto land = [&](int t) {  // after this wave's wait for tile t: zero its chunks past K
    if (ragged && t == nk - 1) {
      float* st = stage(t);
      pa.fix(t, krel, st, wave, lane);
      pb.fix(t, krel, st + PA::FLOATS, wave, lane);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  auto read_frags = [&](int t, float (&a)[FM][8], float (&b)[FN][8]) {
    const float* st = stage(t);
#pragma unroll
    for (int i = 0; i < FM; ++i) pa.frag(st, wm0 + i * 16, l16, kq, a[i]);
#pragma unroll
    for (int j = 0; j < FN; ++j) pb.frag(st + PA::FLOATS, wn0 + j * 16, l16, kq, b[j]);
  };
  auto mfma_step = [&](const float (&a)[FM][8], const float (&b)[FN][8], int s) {
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

  // prologue: tiles 0 .. NB-2 in flight, wait for tile 0
#pragma unroll
  for (int t = 0; t < NB - 1; ++t)
    if (t < nk) issue(t);
  if (nk >= NB - 1) wait_vm<G * (NB - 2)>();
  else wait_vm<0>();
  land(0);
  float a[FM][8], b[FN][8], a1[FM][8], b1[FN][8];
  read_frags(0, a, b);

  auto iteration = [&](int t, float (&ca)[FM][8], float (&cb)[FN][8], float (&na)[FM][8],
                       float (&nb)[FN][8]) {
    const bool more = t + NB - 1 < nk;
    mfma_step(ca, cb, 0);
    mfma_step(ca, cb, 1);
    __builtin_amdgcn_sched_barrier(0);
    if (more) issue(t + NB - 1);  // after the fragments landed (no exposed lgkm wait)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 2; s < 7; ++s) mfma_step(ca, cb, s);
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nk) {
      if (more) wait_vm<G * (NB - 2)>();
      else wait_vm<0>();
      land(t + 1);
      read_frags(t + 1, na, nb);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_step(ca, cb, 7);
  };
  for (int t = 0; t < nk; t += 2) {
    iteration(t, a, b, a1, b1);
    if (t + 1 >= nk) break;
    iteration(t + 1, a1, b1, a, b);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
  }
  finish_tile<BM, BN, WGM, WGN, RS>(p, acc, rs, tile, split, tn, m0, n0, smem);
}

template <int BM, int BN, int WGM, int WGN, int NB, int KINDS>
__device__ __forceinline__ void g3_group_body(const GemmGroup& g, int b, float* smem) {
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
    if (kind == 0) return ring_body<BM, BN, WGM, WGN, true, true, false, NB>(p, lb, smem);
  if constexpr ((KINDS & 2) != 0)
    if (kind == 1) return ring_body<BM, BN, WGM, WGN, true, false, false, NB>(p, lb, smem);
  if constexpr ((KINDS & 4) != 0)
    if (kind == 2) return ring_body<BM, BN, WGM, WGN, false, false, false, NB>(p, lb, smem);
  if constexpr ((KINDS & 8) != 0)
    if (kind == 3) return ring_body<BM, BN, WGM, WGN, false, true, false, NB>(p, lb, smem);
  if constexpr ((KINDS & 16) != 0)
    if (kind == 4) return ring_body<BM, BN, WGM, WGN, false, false, true, NB>(p, lb, smem);
}

template <int BM, int BN, int WGM, int WGN, int OCC, int NB, int KINDS>
__global__ __launch_bounds__(WGM * WGN * 64, OCC) void g3_kernel(const GemmGroup g) {
  __shared__ __attribute__((aligned(16))) float smem[ring_smem_floats<BM, BN, NB>()];
  g3_group_body<BM, BN, WGM, WGN, NB, KINDS>(g, blockIdx.x, smem);
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
  if constexpr (PRIO >= 10)  // body3, PRIO - 10 = ring depth
    hipLaunchKernelGGL((g3_kernel<BM, BN, WGM, WGN, OCC, PRIO - 10, KINDS>), grid, block, 0, st, g);
  else if constexpr (OLD)
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
    case 110: return lab_launch<32, 32, 2, 2, 4, 0, true>(n, d, pl, ws, ws_bytes, st);
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
    // body3 (LDS-DMA ring): 3xx = tile, last digit = ring depth
    case 302: return lab_launch<64, 32, 2, 2, 2, 12, false>(n, d, pl, ws, ws_bytes, st);
    case 303: return lab_launch<64, 32, 2, 2, 2, 13, false>(n, d, pl, ws, ws_bytes, st);
    case 304: return lab_launch<64, 32, 2, 2, 2, 14, false>(n, d, pl, ws, ws_bytes, st);
    case 313: return lab_launch<64, 64, 2, 2, 2, 13, false>(n, d, pl, ws, ws_bytes, st);
    case 314: return lab_launch<64, 64, 2, 2, 2, 14, false>(n, d, pl, ws, ws_bytes, st);
    case 322: return lab_launch<128, 64, 2, 2, 1, 12, false>(n, d, pl, ws, ws_bytes, st);
    case 323: return lab_launch<128, 64, 2, 2, 1, 13, false>(n, d, pl, ws, ws_bytes, st);
    case 324: return lab_launch<128, 64, 2, 2, 1, 14, false>(n, d, pl, ws, ws_bytes, st);
    case 333: return lab_launch<128, 128, 2, 2, 1, 13, false>(n, d, pl, ws, ws_bytes, st);
    case 343: return lab_launch<256, 64, 4, 2, 1, 13, false>(n, d, pl, ws, ws_bytes, st);
    case 353: return lab_launch<64, 128, 2, 2, 1, 13, false>(n, d, pl, ws, ws_bytes, st);
    default: return -3;
  }
}
