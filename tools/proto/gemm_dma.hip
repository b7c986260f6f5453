// PROTOTYPE (r03 A/B; NOT part of libdlrm_hip.so): the exact-f32 MFMA GEMM body with its
// operand panels moved global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) through an
// S-stage ring, instead of global -> registers -> ds_write with one tile of prefetch.
// Question (tools/dma_probe.py): is the production body (gemm.hip pipe_body) bounded by
// its one-tile prefetch / staging instructions?
//
// LDS images, filled 1 KiB (64 lanes x 16 B) per wave instruction:
//   KC  (X(mn, k) = X[mn*ld + k]): 8 rows x 32 k per KiB block; row r's 16-B chunk c sits in
//       slot 8 (r % 8) + (c ^ s(r)), s(r) = (r ^ (r >> 3)) & 7 -> fragment reads
//       (ds_read_b128, lane = row l%16, chunks 2(l/16), 2(l/16)+1) are conflict-free;
//   !KC (X(mn, k) = X[k*ld + mn]): 256/MN k-rows x MN per block; chunk c of row k in slot
//       (k % rpb) (MN/4) + (c ^ g(k)), g(k) = 4 ((k >> 3) & 1) -> ds_read_b32 reads of a
//       column for k = 8 kq + s are conflict-free.
// (bank maps checked offline: every ds_read group touches 64 distinct banks)
#include "common.hpp"  // (dlrm-yx_amd/csrc)

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kBK = 32;
typedef __attribute__((address_space(3))) void lds_void;

template <int MN, bool KC>
struct DImg {
  static constexpr int FLOATS = MN * kBK;            // one stage
  static constexpr int BLOCKS = FLOATS * 4 / 1024;   // KiB blocks (one DMA instr each)
  static constexpr int CPR = MN / 4;                 // !KC: chunks per k-row
  static constexpr int RPB = KC ? 8 : 256 / MN;      // rows per block
  __device__ __forceinline__ static int swz(int r) { return (r ^ (r >> 3)) & 7; }
  __device__ __forceinline__ static int g(int k) { return (4 * ((k >> 3) & 1)) % CPR; }
  // (mn, k of the chunk start) loaded by lane l of block b
  __device__ __forceinline__ static void lane_src(int b, int l, int& mn, int& k) {
    if constexpr (KC) {
      const int r = b * 8 + (l >> 3);
      mn = r;
      k = 4 * ((l & 7) ^ swz(r));
    } else {
      const int kk = b * RPB + l / CPR;
      k = kk;
      mn = 4 * ((l % CPR) ^ g(kk));
    }
  }
  // float offset of element (mn, k) in the stage image
  __device__ __forceinline__ static int at(int mn, int k) {
    if constexpr (KC) {
      const int c = k >> 2;
      return (mn >> 3) * 256 + ((mn & 7) * 8 + (c ^ swz(mn))) * 4 + (k & 3);
    } else {
      const int c = mn >> 2;
      return (k / RPB) * 256 + ((k % RPB) * CPR + (c ^ g(k))) * 4 + (mn & 3);
    }
  }
};

struct PD {
  int64_t M, N, K;
  float alpha;
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int tiles_n;
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8;
  const int q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// One LDS-DMA wave instruction (64 lanes x 16 B -> LDS [lds_addr, +1 KiB)) in inline asm:
// the compiler's waitcnt pass does not see it as an LDS store, so it does not drain every
// in-flight DMA (vmcnt(0)) before the next ds_read of ANOTHER stage; wait_vm<N> orders.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const float* lds_ptr, int voff) {
  const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)lds_ptr;
  asm volatile(
      "s_mov_b32 m0, %0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(a),
      "v"(voff), "s"(r)
      : "memory");  // (m0 is reserved: the compiler never keeps a value in it here)
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, bool A_KC, bool B_KC, int S, bool PIPE>
__global__ __launch_bounds__(256, 2) void gemm_dma_kernel(const PD p) {
  constexpr int WGM = 2, WGN = 2;
  constexpr int WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
  constexpr int KL = kBK / 4;
  using IA = DImg<BM, A_KC>;
  using IB = DImg<BN, B_KC>;
  constexpr int STAGE = IA::FLOATS + IB::FLOATS;
  constexpr int NIA = IA::BLOCKS / 4, NIB = IB::BLOCKS / 4;  // DMA instrs per wave per tile
  static_assert(IA::BLOCKS % 4 == 0 && IB::BLOCKS % 4 == 0, "blocks per wave");
  constexpr int NI = NIA + NIB;
  __shared__ __attribute__((aligned(1024))) float lds[S * STAGE];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - (tile / p.tiles_n) * p.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, l16 = lane & 15;
  const int wm0 = (wave / WGN) * WM, wn0 = (wave % WGN) * WN;
  const int nk = (int)((p.K + kBK - 1) / kBK);

  const int64_t a_ext = A_KC ? (p.M - 1) * p.lda + p.K : (p.K - 1) * p.lda + p.M;
  const int64_t b_ext = B_KC ? (p.N - 1) * p.ldb + p.K : (p.K - 1) * p.ldb + p.N;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)(a_ext * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)(b_ext * 4), 0x00020000);
  // per DMA instruction of this wave: byte offset at K-tile 0 (or -1: row out of range),
  // the chunk's k within the tile
  int aoff[NIA], akp[NIA], boff[NIB], bkp[NIB];
#pragma unroll
  for (int i = 0; i < NIA; ++i) {
    int mn, k;
    IA::lane_src(wave * NIA + i, lane, mn, k);
    const int64_t gmn = m0 + mn;
    aoff[i] = gmn < p.M ? (int)(4 * (A_KC ? gmn * p.lda + k : (int64_t)k * p.lda + gmn)) : -1;
    akp[i] = k;
  }
#pragma unroll
  for (int i = 0; i < NIB; ++i) {
    int mn, k;
    IB::lane_src(wave * NIB + i, lane, mn, k);
    const int64_t gmn = n0 + mn;
    boff[i] = gmn < p.N ? (int)(4 * (B_KC ? gmn * p.ldb + k : (int64_t)k * p.ldb + gmn)) : -1;
    bkp[i] = k;
  }
  const int a_step = A_KC ? 4 * kBK : (int)(4 * kBK * p.lda);
  const int b_step = B_KC ? 4 * kBK : (int)(4 * kBK * p.ldb);
  const int K32 = (int)p.K;
  auto issue = [&](int t) {  // DMA of K-tile t into stage t % S (t < nk + S: zeros past K)
    float* st = lds + (t % S) * STAGE;
#pragma unroll
    for (int i = 0; i < NIA; ++i) {
      const bool ok = aoff[i] >= 0 && t * kBK + akp[i] < K32;
      const int off = ok ? aoff[i] + t * a_step : 0x7ffffff0;
      dma16(ra, st + (wave * NIA + i) * 256, off);
    }
#pragma unroll
    for (int i = 0; i < NIB; ++i) {
      const bool ok = boff[i] >= 0 && t * kBK + bkp[i] < K32;
      const int off = ok ? boff[i] + t * b_step : 0x7ffffff0;
      dma16(rb, st + IA::FLOATS + (wave * NIB + i) * 256, off);
    }
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (PIPE) {
    // fragments of tile t+1 are read (all k-steps) under the second half of tile t's MFMAs
    static_assert(S >= 3, "PIPE needs tile t+1 landed while tile t computes");
    float ca[FM][KL], cb[FN][KL], na[FM][KL], nb[FN][KL];
    auto read = [&](int t, float (&a)[FM][KL], float (&b)[FN][KL]) {
      const float* st = lds + (t % S) * STAGE;
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
      for (int s = s0; s < s1; ++s)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    };
#pragma unroll
    for (int t = 0; t < S - 1; ++t) issue(t);
    wait_vm<(S - 2) * NI>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0, ca, cb);
    auto step = [&](int t, float (&a)[FM][KL], float (&b)[FN][KL], float (&a2)[FM][KL],
                    float (&b2)[FN][KL]) {
      mfma(a, b, 0, KL / 2);
      wait_vm<(S - 3) * NI>();  // tile t+1 landed (this wave)
      __builtin_amdgcn_s_barrier();  // (every wave; tile t-1's stage is free)
      asm volatile("" ::: "memory");
      issue(t + S - 1);
      read(t + 1, a2, b2);
      mfma(a, b, KL / 2, KL);
    };
    for (int t = 0; t < nk; t += 2) {
      step(t, ca, cb, na, nb);
      if (t + 1 >= nk) break;
      step(t + 1, na, nb, ca, cb);
    }
  } else {
#pragma unroll
  for (int t = 0; t < S - 1; ++t) issue(t);
  for (int t = 0; t < nk; ++t) {
    wait_vm<(S - 2) * NI>();  // this wave's DMA of tile t has landed
    // every wave's has; every wave is done with tile t-1's stage.  A bare s_barrier: the
    // fence of __syncthreads would drain every in-flight DMA (vmcnt(0)).
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(t + S - 1);         // into tile t-1's stage
    const float* st = lds + (t % S) * STAGE;
    float a[FM][KL], b[FN][KL];
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
#pragma unroll
    for (int s = 0; s < KL; ++s)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  }
  }
  wait_vm<0>();  // the trailing zero-DMAs (tiles >= nk) before the workgroup's LDS goes away
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

}  // namespace

// C[M][N] = alpha op(A) op(B), fp32 (layout 0: A, B k-contiguous; 1: A k-contig, B stored
// [K][N]; 2: A stored [K][M], B [K][N]); tile 0: 64x64, 1: 64x32; stages 3 or 4.
extern "C" int dlrm_dma_gemm(int32_t layout, int32_t tile, int32_t stages, int64_t M, int64_t N,
                             int64_t K, float alpha, const float* A, int64_t lda, const float* B,
                             int64_t ldb, float* C, int64_t ldc, dlrm_stream_t stream) {
  DLRM_ARG(M > 0 && N > 0 && K > 0 && K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && A && B && C,
           "dlrm_dma_gemm: bad arguments");
  hipStream_t st = dlrm::as_stream(stream);
  PD p{M, N, K, alpha, A, lda, B, ldb, C, ldc, 0};
#define GO(BM, BN, S, PP)                                                                      \
  do {                                                                                         \
    p.tiles_n = (int)dlrm::ceil_div(N, BN);                                                    \
    const dim3 g((unsigned)(dlrm::ceil_div(M, BM) * p.tiles_n));                               \
    if (layout == 0) hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, true, true, S, PP>), g, dim3(256), 0, st, p); \
    else if (layout == 1) hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, true, false, S, PP>), g, dim3(256), 0, st, p); \
    else hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, false, false, S, PP>), g, dim3(256), 0, st, p); \
  } while (0)
  const bool pp = stages >= 10;  // 13 / 14: the fragment-pipelined body with 3 / 4 stages
  stages %= 10;
  if (tile == 1) {
    if (pp) { if (stages == 3) GO(64, 32, 3, true); else GO(64, 32, 4, true); }
    else { if (stages == 3) GO(64, 32, 3, false); else GO(64, 32, 4, false); }
  } else {
    if (pp) { if (stages == 3) GO(64, 64, 3, true); else GO(64, 64, 4, true); }
    else { if (stages == 3) GO(64, 64, 3, false); else GO(64, 64, 4, false); }
  }
#undef GO
  DLRM_LAUNCH_CHECK("dlrm_dma_gemm");
  return DLRM_OK;
}
