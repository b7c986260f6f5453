// PROTOTYPE (r03 A/B; NOT part of libdlrm_hip.so): fp32 GEMM on the bf16 matrix core from
// PRE-SPLIT operands.  Each fp32 operand X arrives as three bf16 planes (h, m, l with
// x = h + m + l, round-to-nearest at each level; dlrm_x6_split_planes writes them), so the
// main loop does no conversion at all: 16-B plane chunks go global -> registers -> LDS
// (the Img6 images of gemm.hip) and each 32-deep K-tile is six v_mfma_f32_16x16x32_bf16
// products per 16x16 output (h*h, h*m, m*h, h*l, l*h, m*m).
//
// Question this answers (tools/x6p_probe.py): with the split moved out of the GEMM, how
// fast is the x6 body on the C3 MLP shapes, against the exact-f32 MFMA body?
// Answer (profiles/r03_x6p_probe.txt): 1.1-1.3x on the big forward / dgrad shapes, so the
// split was never the bound; the body is latency-bound per 32-deep K-tile like the fp32
// one.  Build: make -C tools/proto  (-> tools/proto/libdlrm_x6p.so, loaded by the probe).
#include "common.hpp"  // (dlrm-yx_amd/csrc)

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using s16x4 = __attribute__((ext_vector_type(4))) short;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int kBK = 32;

__device__ __forceinline__ unsigned pk_bf16(float x0, float x1) {
  using bf16x2 = __attribute__((ext_vector_type(2))) __bf16;
  return __builtin_bit_cast(unsigned, bf16x2{(__bf16)x0, (__bf16)x1});
}
__device__ __forceinline__ float lo_f(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float hi_f(unsigned u) {
  return __builtin_bit_cast(float, u & 0xffff0000u);
}
__device__ __forceinline__ void split2(float x0, float x1, unsigned& h, unsigned& m,
                                       unsigned& l) {
  h = pk_bf16(x0, x1);
  const float r0 = x0 - lo_f(h), r1 = x1 - hi_f(h);
  m = pk_bf16(r0, r1);
  const float s0 = r0 - lo_f(m), s1 = r1 - hi_f(m);
  l = pk_bf16(s0, s1);
}

// Three-plane bf16 LDS image of one operand's (MN x 32) panel (gemm.hip Img6).
template <int MN, bool KC>
struct Img {
  static constexpr int BK = kBK;
  static constexpr int PITCH = KC ? BK + 8 : MN + 16;
  static constexpr int OCT = 8 * PITCH + 64;
  static constexpr int PLANE = KC ? MN * PITCH : (BK / 8) * OCT;
  static constexpr int SIZE = 3 * PLANE;
  // 16-B chunks per K-tile: KC (plane, mn, k octet), !KC (plane, k, mn octet)
  static constexpr int CHUNKS = 3 * MN * BK / 8;

  __device__ __forceinline__ static void chunk_coords(int c, int& q, int& mn, int& k) {
    if constexpr (KC) {
      q = c / (MN * 4);
      const int r = c - q * MN * 4;
      mn = r >> 2;
      k = 8 * (r & 3);
    } else {
      q = c / (MN * BK / 8);
      const int r = c - q * (MN * BK / 8);
      k = r / (MN / 8);
      mn = 8 * (r - k * (MN / 8));
    }
  }
  __device__ __forceinline__ static int lds_off(int q, int mn, int k) {
    return q * PLANE + (KC ? mn * PITCH + k : (k >> 3) * OCT + (k & 7) * PITCH + mn);
  }
  __device__ __forceinline__ static bf16x8 frag(const __bf16* buf, int q, int mn0, int l16,
                                                int kq) {
    const __bf16* pl = buf + q * PLANE;
    if constexpr (KC) {
      return __builtin_bit_cast(
          bf16x8, *reinterpret_cast<const uint4*>(pl + (mn0 + l16) * PITCH + kq * 8));
    } else {
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

struct P6 {
  int64_t M, N, K;
  float alpha;
  const __bf16* A;  // planes of op(A): KC [3][M][lda] / !KC [3][K][lda]
  int64_t lda, psa;
  const __bf16* B;  // planes of op(B): KC [3][N][ldb] / !KC [3][K][ldb]
  int64_t ldb, psb;
  float* C;
  int64_t ldc;
  int tiles_n;
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8;
  const int q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <int BM, int BN, bool A_KC, bool B_KC>
__global__ __launch_bounds__(256, 1) void gemm6p_kernel(const P6 p) {
  constexpr int NT = 256, WGM = 2, WGN = 2;
  constexpr int WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
  using IA = Img<BM, A_KC>;
  using IB = Img<BN, B_KC>;
  constexpr int BUF = IA::SIZE + IB::SIZE;
  constexpr int CA = IA::CHUNKS / NT, CB = IB::CHUNKS / NT;
  static_assert(IA::CHUNKS % NT == 0 && IB::CHUNKS % NT == 0, "chunk map");
  constexpr int NS = CA + CB;
  constexpr int NP = 6;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * BUF];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - (tile / p.tiles_n) * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, l16 = lane & 15;
  const int wm0 = (wave / WGN) * WM, wn0 = (wave % WGN) * WN;

  // raw buffer descriptors over the planes (OOB chunks read as zeros)
  const int64_t a_ext = 2 * p.psa + (A_KC ? p.M * p.lda : p.K * p.lda);
  const int64_t b_ext = 2 * p.psb + (B_KC ? p.N * p.ldb : p.K * p.ldb);
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)(a_ext * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)(b_ext * 2), 0x00020000);
  // per-chunk byte offsets at K-tile 0, LDS offsets, validity
  int goff[NS], loff[NS], kpos[NS];
  bool ok[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c) {
    int q, mn, k;
    if (c < CA) {
      IA::chunk_coords(tid + c * NT, q, mn, k);
      const int64_t gmn = m0 + mn;
      goff[c] = (int)(2 * (q * p.psa + (A_KC ? gmn * p.lda + k : (int64_t)k * p.lda + gmn)));
      ok[c] = gmn < p.M;
      kpos[c] = k;
      loff[c] = IA::lds_off(q, mn, k);
    } else {
      IB::chunk_coords(tid + (c - CA) * NT, q, mn, k);
      const int64_t gmn = n0 + mn;
      goff[c] = (int)(2 * (q * p.psb + (B_KC ? gmn * p.ldb + k : (int64_t)k * p.ldb + gmn)));
      ok[c] = gmn < p.N;
      kpos[c] = k;
      loff[c] = IA::SIZE + IB::lds_off(q, mn, k);
    }
  }
  const int a_step = A_KC ? 2 * kBK : (int)(2 * kBK * p.lda);
  const int b_step = B_KC ? 2 * kBK : (int)(2 * kBK * p.ldb);
  const int nk = (int)((p.K + kBK - 1) / kBK);
  uint4 st[NS];
  auto fetch = [&](int c, int t) {
    const bool kc = c < CA ? A_KC : B_KC;
    // KC: the chunk's k must be < K; !KC: its row k must be < K (K % 8 == 0: host check)
    const bool live = ok[c] && t * kBK + kpos[c] < p.K;
    const int off = live ? goff[c] + t * (c < CA ? a_step : b_step) : 0x7ffffff0;
    (void)kc;
    st[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(c < CA ? ra : rb, off,
                                                                            0, 0));
  };
  auto put = [&](int c, __bf16* buf) { *reinterpret_cast<uint4*>(buf + loff[c]) = st[c]; };

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
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
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

  Frag a[FM], b[FN], a1[FM], b1[FN];
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch(c, 0);
#pragma unroll
  for (int c = 0; c < NS; ++c) put(c, lds);
#pragma unroll
  for (int c = 0; c < NS; ++c) fetch(c, 1);
  __syncthreads();
  read_frags(lds, a, b);

  // NS chunk puts / fetches spread over the first NP-1 product steps
  constexpr int PER = (NS + NP - 2) / (NP - 1);
  auto iteration = [&](int kt, const Frag (&ca)[FM], const Frag (&cb)[FN], Frag (&na)[FM],
                       Frag (&nb)[FN]) {
    __bf16* nbuf = lds + ((kt + 1) & 1) * BUF;
#pragma unroll
    for (int s = 0; s < NP - 1; ++s) {
      products(s, ca, cb);
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int c = s * PER + u;
        if (c < NS) {
          put(c, nbuf);
          fetch(c, kt + 2);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    read_frags(nbuf, na, nb);
    __builtin_amdgcn_sched_barrier(0);
    products(NP - 1, ca, cb);
  };
  for (int kt = 0; kt < nk; kt += 2) {
    iteration(kt, a, b, a1, b1);
    if (kt + 1 >= nk) break;
    iteration(kt + 1, a1, b1, a, b);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = n0 + wn0 + j * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm0 + i * 16 + 4 * kq + r;
        if (row < p.M && col < p.N) p.C[row * p.ldc + col] = p.alpha * acc[i][j][r];
      }
    }
}


// ---- DMA-ring variant (r03 probe 2): planes go global -> LDS by buffer_load ... lds through
// an S-stage ring (S-1 K-tiles in flight, no staging registers, no ds_write); swizzled images
// (tools: bank check in DESIGN) read by ds_read_b128 (KC) / ds_read_b64_tr_b16 (!KC).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const void* lds, int voff) {
  const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)lds;
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(a),
               "v"(voff), "s"(r)
               : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int MN, bool KC>
struct DI6 {
  static constexpr int SLOTS = 4 * MN;    // 16-B slots per plane-stage (MN x 32 bf16)
  static constexpr int BYTES = 16 * SLOTS;
  static constexpr int CPR = MN / 8;      // !KC: chunks per k-row
  static constexpr int BLK = SLOTS / 64;  // 1-KiB DMA blocks per plane
  __device__ __forceinline__ static int swk(int r) { return (r >> 1) & 3; }
  __device__ __forceinline__ static int swt(int k) {
    return ((CPR >= 16 ? 2 : 1) * (k ^ (k >> 1))) % CPR;
  }
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
  // fragment of 16 rows/cols at mn0 for lane (l16, kq): 8 bf16 along k
  __device__ __forceinline__ static bf16x8 frag(const char* plane, int mn0, int l16, int kq) {
    if constexpr (KC) {
      const int r = mn0 + l16;
      return __builtin_bit_cast(
          bf16x8, *reinterpret_cast<const uint4*>(plane + 16 * (4 * r + (kq ^ swk(r)))));
    } else {
      const int q = l16 >> 2, p = l16 & 3;
      const int ch = mn0 / 8 + (p >> 1);
      const int k0 = 8 * kq + q, k1 = k0 + 4;
      const char* a0 = plane + 16 * (k0 * CPR + (ch ^ swt(k0))) + 8 * (p & 1);
      const char* a1 = plane + 16 * (k1 * CPR + (ch ^ swt(k1))) + 8 * (p & 1);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
      using s16x8 = __attribute__((ext_vector_type(8))) short;
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

template <int BM, int BN, bool A_KC, bool B_KC, int S>
__global__ __launch_bounds__(256, 1) void gemm6d_kernel(const P6 p) {
  constexpr int WGM = 2, WGN = 2, NW = 4;
  constexpr int WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
  using IA = DI6<BM, A_KC>;
  using IB = DI6<BN, B_KC>;
  constexpr int STAGE = 3 * (IA::BYTES + IB::BYTES);
  constexpr int NBA = 3 * IA::BLK, NBB = 3 * IB::BLK;
  static_assert(NBA % NW == 0 && NBB % NW == 0, "blocks per wave");
  constexpr int NIA = NBA / NW, NIB = NBB / NW, NI = NIA + NIB;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - (tile / p.tiles_n) * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, l16 = lane & 15;
  const int wm0 = (wave / WGN) * WM, wn0 = (wave % WGN) * WN;
  const int64_t a_ext = 2 * p.psa + (A_KC ? p.M * p.lda : p.K * p.lda);
  const int64_t b_ext = 2 * p.psb + (B_KC ? p.N * p.ldb : p.K * p.ldb);
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)(a_ext * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)(b_ext * 2), 0x00020000);
  int aoff[NIA], akp[NIA], boff[NIB], bkp[NIB];
#pragma unroll
  for (int i = 0; i < NIA; ++i) {
    const int b = wave * NIA + i;
    const int q = b / IA::BLK, bb = b % IA::BLK;
    int mn, k;
    IA::src(bb * 64 + lane, mn, k);
    const int64_t g = m0 + mn;
    aoff[i] = g < p.M ? (int)(2 * (q * p.psa + (A_KC ? g * p.lda + k : (int64_t)k * p.lda + g)))
                      : -1;
    akp[i] = k;
  }
#pragma unroll
  for (int i = 0; i < NIB; ++i) {
    const int b = wave * NIB + i;
    const int q = b / IB::BLK, bb = b % IB::BLK;
    int mn, k;
    IB::src(bb * 64 + lane, mn, k);
    const int64_t g = n0 + mn;
    boff[i] = g < p.N ? (int)(2 * (q * p.psb + (B_KC ? g * p.ldb + k : (int64_t)k * p.ldb + g)))
                      : -1;
    bkp[i] = k;
  }
  const int a_step = A_KC ? 2 * kBK : (int)(2 * kBK * p.lda);
  const int b_step = B_KC ? 2 * kBK : (int)(2 * kBK * p.ldb);
  const int K32 = (int)p.K;
  const int nk = (K32 + kBK - 1) / kBK;
  auto issue = [&](int t) {
    char* st = smem + (t % S) * STAGE;
#pragma unroll
    for (int i = 0; i < NIA; ++i) {
      const int b = wave * NIA + i;
      const bool ok = aoff[i] >= 0 && t * kBK + akp[i] < K32;
      dma16(ra, st + (b / IA::BLK) * IA::BYTES + (b % IA::BLK) * 1024,
            ok ? aoff[i] + t * a_step : 0x7ffffff0);
    }
#pragma unroll
    for (int i = 0; i < NIB; ++i) {
      const int b = wave * NIB + i;
      const bool ok = boff[i] >= 0 && t * kBK + bkp[i] < K32;
      dma16(rb, st + 3 * IA::BYTES + (b / IB::BLK) * IB::BYTES + (b % IB::BLK) * 1024,
            ok ? boff[i] + t * b_step : 0x7ffffff0);
    }
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
  auto products = [&](int s0, int s1, const Frag (&ca)[FM], const Frag (&cb)[FN]) {
    constexpr int PA[6] = {0, 2, 1, 0, 1, 0};
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
  Frag ca[FM], cb[FN], na[FM], nb[FN];
#pragma unroll
  for (int t = 0; t < S - 1; ++t) issue(t);
  wait_vm<(S - 2) * NI>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read(0, ca, cb);
  auto step = [&](int t, const Frag (&a)[FM], const Frag (&b)[FN], Frag (&a2)[FM],
                  Frag (&b2)[FN]) {
    products(0, 3, a, b);
    wait_vm<(S - 3) * NI>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(t + S - 1);
    read(t + 1, a2, b2);
    products(3, 6, a, b);
  };
  for (int t = 0; t < nk; t += 2) {
    step(t, ca, cb, na, nb);
    if (t + 1 >= nk) break;
    step(t + 1, na, nb, ca, cb);
  }
  wait_vm<0>();
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = n0 + wn0 + j * 16 + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm0 + i * 16 + 4 * kq + r;
        if (row < p.M && col < p.N) p.C[row * p.ldc + col] = p.alpha * acc[i][j][r];
      }
    }
}

// X [rows][cols] fp32 (ld) -> planes [3][rows][ldp] bf16 (plane stride ps), 8 per thread.
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ X,
                                                           int64_t rows, int64_t cols,
                                                           int64_t ld, __bf16* __restrict__ P,
                                                           int64_t ldp, int64_t ps) {
  const int64_t c8 = (cols + 7) / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * c8) return;
  const int64_t r = i / c8, c = 8 * (i - (i / c8) * c8);
  float x[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = (c + u < cols) ? X[r * ld + c + u] : 0.f;
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) split2(x[2 * u], x[2 * u + 1], h[u], m[u], l[u]);
  __bf16* dst = P + r * ldp + c;
  *reinterpret_cast<uint4*>(dst) = make_uint4(h[0], h[1], h[2], h[3]);
  *reinterpret_cast<uint4*>(dst + ps) = make_uint4(m[0], m[1], m[2], m[3]);
  *reinterpret_cast<uint4*>(dst + 2 * ps) = make_uint4(l[0], l[1], l[2], l[3]);
}

}  // namespace

extern "C" int dlrm_x6_split_planes(const float* X, int64_t rows, int64_t cols, int64_t ld,
                                    void* planes, int64_t ldp, int64_t plane_stride,
                                    dlrm_stream_t stream) {
  DLRM_ARG(X && planes && rows >= 0 && cols >= 0 && ldp % 8 == 0 && ldp >= (cols + 7) / 8 * 8,
           "dlrm_x6_split_planes: bad arguments");
  const int64_t n = rows * ((cols + 7) / 8);
  if (n == 0) return DLRM_OK;
  hipLaunchKernelGGL(split_planes_kernel, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), X, rows, cols, ld, static_cast<__bf16*>(planes),
                     ldp, plane_stride);
  DLRM_LAUNCH_CHECK("dlrm_x6_split_planes");
  return DLRM_OK;
}

// C[M][N] = alpha * op(A) op(B) from planes (layout: 0 A,B KC; 1 A KC, B !KC; 2 A,B !KC).
extern "C" int dlrm_x6p_gemm(int32_t layout, int32_t tile, int64_t M, int64_t N, int64_t K,
                             float alpha, const void* Ap, int64_t lda, int64_t psa,
                             const void* Bp, int64_t ldb, int64_t psb, float* C, int64_t ldc,
                             dlrm_stream_t stream) {
  DLRM_ARG(M > 0 && N > 0 && K > 0 && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && Ap && Bp && C,
           "dlrm_x6p_gemm: bad arguments");
  hipStream_t st = dlrm::as_stream(stream);
  P6 p{M, N, K, alpha, static_cast<const __bf16*>(Ap), lda, psa,
       static_cast<const __bf16*>(Bp), ldb, psb, C, ldc, 0};
#define GO(BM, BN)                                                                            \
  do {                                                                                        \
    p.tiles_n = (int)dlrm::ceil_div(N, BN);                                                   \
    const dim3 g((unsigned)(dlrm::ceil_div(M, BM) * p.tiles_n));                              \
    if (layout == 0) hipLaunchKernelGGL((gemm6p_kernel<BM, BN, true, true>), g, dim3(256), 0, st, p); \
    else if (layout == 1) hipLaunchKernelGGL((gemm6p_kernel<BM, BN, true, false>), g, dim3(256), 0, st, p); \
    else hipLaunchKernelGGL((gemm6p_kernel<BM, BN, false, false>), g, dim3(256), 0, st, p); \
  } while (0)
#define GOD(BM, BN, S)                                                                        \
  do {                                                                                        \
    p.tiles_n = (int)dlrm::ceil_div(N, BN);                                                   \
    const dim3 g((unsigned)(dlrm::ceil_div(M, BM) * p.tiles_n));                              \
    const size_t sm = (size_t)S * 3 * 64 * (BM + BN);                                         \
    if (layout == 0) { (void)hipFuncSetAttribute((const void*)gemm6d_kernel<BM, BN, true, true, S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm); hipLaunchKernelGGL((gemm6d_kernel<BM, BN, true, true, S>), g, dim3(256), sm, st, p); } \
    else if (layout == 1) { (void)hipFuncSetAttribute((const void*)gemm6d_kernel<BM, BN, true, false, S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm); hipLaunchKernelGGL((gemm6d_kernel<BM, BN, true, false, S>), g, dim3(256), sm, st, p); } \
    else { (void)hipFuncSetAttribute((const void*)gemm6d_kernel<BM, BN, false, false, S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm); hipLaunchKernelGGL((gemm6d_kernel<BM, BN, false, false, S>), g, dim3(256), sm, st, p); } \
  } while (0)
  if (tile == 2) GO(128, 64);
  else if (tile == 3) GOD(128, 64, 4);
  else if (tile == 4) GOD(64, 64, 4);
  else if (tile == 5) GOD(64, 64, 3);
  else GO(64, 64);
#undef GO
#undef GOD
  DLRM_LAUNCH_CHECK("dlrm_x6p_gemm");
  return DLRM_OK;
}
