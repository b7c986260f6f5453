// Table-batched EmbeddingBag (sum pooling) for gfx950: forward gather-reduce and
// deterministic sorted backward with the optimizer fused in.
//
// Semantics follow nn.EmbeddingBag(mode="sum") as DLRM_Net.apply_emb calls it
// (dlrm_s_pytorch.py:526-587) in the table-batched CSR layout of
// dlrm_data_pytorch.py:748-753 / TableBatchedEmbeddingBags (dlrm_s_pytorch.py:321-334):
// bag (t, b) = t*B + b owns lookups [offsets[bag], offsets[bag+1]).
//
// Design (MI355X-first, not a translation of yx_modfs/table_batched_embeddings_cuda_yx.cu):
//  * one lane-group of LPB lanes per bag (LPB = D/4 rounded to a power of two, <= 64),
//    64/LPB bags per wave64, so a D=128 row is one coalesced 512-B float4 sweep by 32 lanes;
//  * the group loads up to LPB indices of its bag in one coalesced load and broadcasts
//    them with wave shuffles (ds_bpermute), four row fetches in flight per lane;
//  * 64-bit row bases (a 54 M x 128 table set is 6.9e9 elements);
//  * backward (tbe_bwd.hip): stable radix sort of (global row, lookup) pairs, fixed
//    blocks of 16 lookups (64 from 2^18 lookups per call) summed per run of equal rows,
//    partials combined in block order; every weight row read and written once — bitwise
//    reproducible.
#include "tbe_common.hpp"

namespace {

// ----------------------------------------------------------------- forward --
template <int LPB, int VW, int MAXV, typename IdxT, typename OffT>
__global__ __launch_bounds__(256) void tbe_fwd_kernel(
    const float* __restrict__ W, int64_t D, const int64_t* __restrict__ row_base, int T, int B,
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, const float* __restrict__ psw,
    float* __restrict__ out, int64_t out_bs, int32_t* __restrict__ err) {
  tbe_fwd_body<LPB, VW, MAXV, IdxT, OffT>(W, D, row_base, T, B, idx, off, psw, out, out_bs, err,
                                          blockIdx.x, gridDim.x);
}

// ------------------------------------------------- sparse-grad expansion ----
template <typename OffT>
__global__ __launch_bounds__(256) void tbe_expand_grad_kernel(int64_t D, int T, int B,
                                                              const OffT* __restrict__ off,
                                                              int64_t N,
                                                              const float* __restrict__ psw,
                                                              const float* __restrict__ gout,
                                                              int64_t gbs,
                                                              float* __restrict__ values) {
  // One wave per lookup; lanes sweep D.
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t nb = (int64_t)T * B;
  for (int64_t p = wave; p < N; p += nw) {
    float* vrow = values + p * D;
    if (p < (int64_t)off[0] || p >= (int64_t)off[nb]) {
      for (int64_t d = lane; d < D; d += 64) vrow[d] = 0.f;
      continue;
    }
    int64_t lo = 0, hi = nb;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)off[mid] <= p)
        lo = mid;
      else
        hi = mid;
    }
    const int t = (int)(lo / B);
    const int b = (int)(lo - (int64_t)t * B);
    const float w = psw ? psw[p] : 1.f;
    const float* grow = gout + (int64_t)b * gbs + (int64_t)t * D;
    for (int64_t d = lane; d < D; d += 64) vrow[d] = psw ? w * grow[d] : grow[d];
  }
}

// ------------------------------------------- per-sample-weight gradient ----
// d loss / d w_l = <grad_out[bag(l)], W[row_base[t] + indices[l]]> for every lookup l (the
// gradient the reference's learned weighted pooling receives through
// per_sample_weights, dlrm_s_pytorch.py:475-478, 544-545).  One wave per lookup, lanes
// sweep D, a fixed-order wave reduction: deterministic.  Lookups outside every bag or with
// an out-of-range index get 0.
template <typename IdxT, typename OffT>
__global__ __launch_bounds__(256) void tbe_psw_grad_kernel(
    const float* __restrict__ W, int64_t D, const int64_t* __restrict__ row_base, int T, int B,
    const IdxT* __restrict__ idx, const OffT* __restrict__ off, int64_t N,
    const float* __restrict__ gout, int64_t gbs, float* __restrict__ gpsw) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t nb = (int64_t)T * B;
  for (int64_t p = wave; p < N; p += nw) {
    float s = 0.f;
    if (p >= (int64_t)off[0] && p < (int64_t)off[nb]) {
      int64_t lo = 0, hi = nb;
      while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)off[mid] <= p)
          lo = mid;
        else
          hi = mid;
      }
      const int t = (int)(lo / B);
      const int b = (int)(lo - (int64_t)t * B);
      const int64_t r = (int64_t)idx[p];
      if (r >= 0 && r < row_base[t + 1] - row_base[t]) {
        const float* wrow = W + (row_base[t] + r) * D;
        const float* grow = gout + (int64_t)b * gbs + (int64_t)t * D;
        for (int64_t d = lane; d < D; d += 64) s = fmaf(wrow[d], grow[d], s);
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if (lane == 0) gpsw[p] = s;
  }
}

// ------------------------------------------------------------------- QR ----
template <typename IdxT>
__global__ __launch_bounds__(256) void qr_split_kernel(const IdxT* __restrict__ idx, int64_t n,
                                                       int64_t c, int64_t* __restrict__ q,
                                                       int64_t* __restrict__ r) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t v = (int64_t)idx[i];
  // (input / num_collisions).long(): true division in fp32, truncated.
  const float qf = (float)v / (float)c;
  q[i] = (int64_t)qf;
  int64_t rr = v % c;  // torch.remainder: sign of the divisor
  if (rr != 0 && ((rr < 0) != (c < 0))) rr += c;
  r[i] = rr;
}

__global__ __launch_bounds__(256) void qr_combine_fwd_kernel(int op, int64_t nrows, int64_t D,
                                                             const float* __restrict__ eq,
                                                             const float* __restrict__ er,
                                                             float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows * D) return;
  if (op == DLRM_QR_MULT) {
    out[i] = eq[i] * er[i];
  } else if (op == DLRM_QR_ADD) {
    out[i] = eq[i] + er[i];
  } else {
    const int64_t m = i / D, d = i - m * D;
    out[m * 2 * D + d] = eq[i];
    out[m * 2 * D + D + d] = er[i];
  }
}

__global__ __launch_bounds__(256) void qr_combine_bwd_kernel(int op, int64_t nrows, int64_t D,
                                                             const float* __restrict__ eq,
                                                             const float* __restrict__ er,
                                                             const float* __restrict__ go,
                                                             float* __restrict__ geq,
                                                             float* __restrict__ ger) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows * D) return;
  if (op == DLRM_QR_MULT) {
    const float g = go[i];
    geq[i] = g * er[i];
    ger[i] = g * eq[i];
  } else if (op == DLRM_QR_ADD) {
    geq[i] = go[i];
    ger[i] = go[i];
  } else {
    const int64_t m = i / D, d = i - m * D;
    geq[i] = go[m * 2 * D + d];
    ger[i] = go[m * 2 * D + D + d];
  }
}

// ------------------------------------------------------------ CSR build ----
struct CsrArgs {
  const int64_t* off[64];
  int64_t start[65];
};

template <typename OutT>
__global__ __launch_bounds__(256) void csr_from_tables_kernel(int T, int B, CsrArgs a,
                                                              OutT* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = (int64_t)T * B;
  if (i > nb) return;
  if (i == nb) {
    out[nb] = (OutT)a.start[T];
    return;
  }
  const int t = (int)(i / B);
  const int b = (int)(i - (int64_t)t * B);
  out[i] = (OutT)(a.start[t] + a.off[t][b]);
}

// ------------------------------------------------------------- dispatch ----
template <typename IdxT, typename OffT>
int launch_fwd(const float* W, int64_t D, const int64_t* row_base, int T, int B, const void* idx,
               const void* off, const float* psw, float* out, int64_t out_bs, int32_t* err,
               hipStream_t st) {
  const bool vec4 = (D % 4 == 0) && ((reinterpret_cast<uintptr_t>(W) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(out) & 15) == 0) && (out_bs % 4 == 0);
  const int64_t nchunks = vec4 ? D / 4 : D;
  int lpb = 1;
  while (lpb < nchunks && lpb < 64) lpb <<= 1;
  const int64_t maxv = dlrm::ceil_div(nchunks, lpb);
  DLRM_REQUIRE(maxv <= 8, DLRM_ERR_UNSUPPORTED, "tbe_forward: D=%lld too large",
               (long long)D);
  const int64_t nbags = (int64_t)T * B;
  const int gpw = 64 / lpb;
  int64_t blocks = dlrm::ceil_div(dlrm::ceil_div(nbags, gpw), 4);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  const IdxT* ip = static_cast<const IdxT*>(idx);
  const OffT* op = static_cast<const OffT*>(off);
#define FWD(LPB, VW, MV)                                                                   \
  hipLaunchKernelGGL((tbe_fwd_kernel<LPB, VW, MV, IdxT, OffT>), dim3(blocks), dim3(256), 0, \
                     st, W, D, row_base, T, B, ip, op, psw, out, out_bs, err)
#define FWD_LPB(VW)                        \
  switch (lpb) {                           \
    case 1: FWD(1, VW, 1); break;          \
    case 2: FWD(2, VW, 1); break;          \
    case 4: FWD(4, VW, 1); break;          \
    case 8: FWD(8, VW, 1); break;          \
    case 16: FWD(16, VW, 1); break;        \
    case 32: FWD(32, VW, 1); break;        \
    default:                               \
      if (maxv == 1) FWD(64, VW, 1);       \
      else if (maxv == 2) FWD(64, VW, 2);  \
      else if (maxv <= 4) FWD(64, VW, 4);  \
      else FWD(64, VW, 8);                 \
  }
  if (vec4) {
    FWD_LPB(4)
  } else {
    FWD_LPB(1)
  }
#undef FWD_LPB
#undef FWD
  DLRM_LAUNCH_CHECK("dlrm_tbe_forward");
  return DLRM_OK;
}

}  // namespace

extern "C" int dlrm_tbe_forward(const float* weights, int64_t D, const int64_t* row_base,
                                int32_t T, int32_t B, const void* indices, int32_t index_bits,
                                const void* offsets, int32_t offset_bits,
                                const float* per_sample_weights, float* out,
                                int64_t out_batch_stride, int32_t* error_flag,
                                dlrm_stream_t stream) {
  DLRM_ARG(weights && row_base && out && offsets, "dlrm_tbe_forward: null pointer");
  DLRM_ARG(T > 0 && B > 0 && D > 0, "dlrm_tbe_forward: bad sizes T=%d B=%d D=%lld", T, B,
           (long long)D);
  DLRM_ARG(index_bits == 32 || index_bits == 64, "dlrm_tbe_forward: index_bits must be 32|64");
  DLRM_ARG(offset_bits == 32 || offset_bits == 64,
           "dlrm_tbe_forward: offset_bits must be 32|64");
  DLRM_ARG(out_batch_stride >= (int64_t)T * D, "dlrm_tbe_forward: out_batch_stride < T*D");
  hipStream_t st = dlrm::as_stream(stream);
  if (index_bits == 32 && offset_bits == 32)
    return launch_fwd<int32_t, int32_t>(weights, D, row_base, T, B, indices, offsets,
                                        per_sample_weights, out, out_batch_stride, error_flag, st);
  if (index_bits == 32)
    return launch_fwd<int32_t, int64_t>(weights, D, row_base, T, B, indices, offsets,
                                        per_sample_weights, out, out_batch_stride, error_flag, st);
  if (offset_bits == 32)
    return launch_fwd<int64_t, int32_t>(weights, D, row_base, T, B, indices, offsets,
                                        per_sample_weights, out, out_batch_stride, error_flag, st);
  return launch_fwd<int64_t, int64_t>(weights, D, row_base, T, B, indices, offsets,
                                      per_sample_weights, out, out_batch_stride, error_flag, st);
}

// Table-batched QR (the fused engine's QR tables): logical CSR -> physical CSR.  Physical
// table p takes logical table src[p]'s bags; its indices are the logical ones (kind 0), the
// quotients (kind 1) or the remainders (kind 2) by coll[p].  Grid: x over the larger of a
// table's lookups and its bags (grid-stride), y = physical table.
template <typename IdxT, typename OffT>
__global__ __launch_bounds__(256) void qr_expand_kernel(
    int T_phys, int B, const IdxT* __restrict__ idx, const OffT* __restrict__ off,
    const int32_t* __restrict__ src, const int32_t* __restrict__ kind,
    const int32_t* __restrict__ coll, int32_t* __restrict__ pidx, int32_t* __restrict__ poff,
    int64_t cap, int32_t* __restrict__ err) {
  const int p = blockIdx.y;
  const int j = src[p];
  const int64_t s = (int64_t)off[(int64_t)j * B];
  const int64_t len = (int64_t)off[(int64_t)(j + 1) * B] - s;
  int64_t base = 0;  // lookups of the physical tables before p
  for (int q = 0; q < p; ++q)
    base += (int64_t)off[(int64_t)(src[q] + 1) * B] - (int64_t)off[(int64_t)src[q] * B];
  const int k = kind[p];
  const int64_t c = coll[p];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t lim = len > B ? len : B;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += stride) {
    if (i < len) {
      const int64_t v = (int64_t)idx[s + i];
      int64_t o = v;
      if (k == 1) {
        o = (int64_t)((float)v / (float)c);  // (input / num_collisions).long()
      } else if (k == 2) {
        o = v % c;  // torch.remainder: sign of the divisor
        if (o != 0 && ((o < 0) != (c < 0))) o += c;
      }
      if (base + i < cap) {
        pidx[base + i] = (int32_t)o;
      } else if (err) {  // past the caller's buffer: dropped (the offsets are clamped)
        atomicOr(err, DLRM_TBE_ERR_TABLE_CAP);
      }
    }
    if (i < B) {
      const int64_t o = base + (int64_t)off[(int64_t)j * B + i] - s;
      poff[(int64_t)p * B + i] = (int32_t)(o < cap ? o : cap);
    }
  }
  if (p == T_phys - 1 && blockIdx.x == 0 && threadIdx.x == 0)
    poff[(int64_t)T_phys * B] = (int32_t)(base + len < cap ? base + len : cap);
}

// E[b][t] = op(P[b][pq[t]], P[b][pr[t]]) for QR tables (pr[t] >= 0), P[b][pq[t]] otherwise.
__global__ __launch_bounds__(256) void qr_pool_fwd_kernel(int op, int T, int64_t B, int64_t D4,
                                                          const int32_t* __restrict__ pq,
                                                          const int32_t* __restrict__ pr,
                                                          const float4* __restrict__ P,
                                                          int64_t pbs4, float4* __restrict__ E,
                                                          int64_t ebs4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per_b = (int64_t)T * D4;
  if (i >= B * per_b) return;
  const int64_t b = i / per_b, r = i - b * per_b, t = r / D4, d = r - t * D4;
  const float4 a = P[b * pbs4 + (int64_t)pq[t] * D4 + d];
  float4 o = a;
  if (pr[t] >= 0) {
    const float4 c = P[b * pbs4 + (int64_t)pr[t] * D4 + d];
    if (op == DLRM_QR_MULT)
      o = make_float4(a.x * c.x, a.y * c.y, a.z * c.z, a.w * c.w);
    else
      o = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, a.w + c.w);
  }
  E[b * ebs4 + t * D4 + d] = o;
}

__global__ __launch_bounds__(256) void qr_pool_bwd_kernel(int op, int T, int64_t B, int64_t D4,
                                                          const int32_t* __restrict__ pq,
                                                          const int32_t* __restrict__ pr,
                                                          const float4* __restrict__ P,
                                                          int64_t pbs4,
                                                          const float4* __restrict__ dE,
                                                          int64_t ebs4, float4* __restrict__ dP,
                                                          int64_t dpbs4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per_b = (int64_t)T * D4;
  if (i >= B * per_b) return;
  const int64_t b = i / per_b, r = i - b * per_b, t = r / D4, d = r - t * D4;
  const float4 g = dE[b * ebs4 + t * D4 + d];
  const int64_t oq = (int64_t)pq[t] * D4 + d;
  if (pr[t] < 0) {
    dP[b * dpbs4 + oq] = g;
    return;
  }
  const int64_t orr = (int64_t)pr[t] * D4 + d;
  if (op == DLRM_QR_MULT) {
    const float4 a = P[b * pbs4 + oq], c = P[b * pbs4 + orr];
    dP[b * dpbs4 + oq] = make_float4(g.x * c.x, g.y * c.y, g.z * c.z, g.w * c.w);
    dP[b * dpbs4 + orr] = make_float4(g.x * a.x, g.y * a.y, g.z * a.z, g.w * a.w);
  } else {
    dP[b * dpbs4 + oq] = g;
    dP[b * dpbs4 + orr] = g;
  }
}

extern "C" int dlrm_qr_expand_csr(int32_t T_phys, int32_t B, const void* indices,
                                  int32_t index_bits, const void* offsets, int32_t offset_bits,
                                  const int32_t* src, const int32_t* kind, const int32_t* coll,
                                  int64_t max_lookups_per_table, int32_t* phys_indices,
                                  int32_t* phys_offsets, int64_t phys_capacity,
                                  int32_t* error_flag, dlrm_stream_t stream) {
  DLRM_ARG(T_phys > 0 && B > 0 && phys_capacity >= 0, "dlrm_qr_expand_csr: bad sizes");
  DLRM_ARG(indices && offsets && src && kind && coll && phys_indices && phys_offsets,
           "dlrm_qr_expand_csr: null pointer");
  DLRM_ARG(index_bits == 32 || index_bits == 64, "dlrm_qr_expand_csr: bad index_bits");
  DLRM_ARG(offset_bits == 32 || offset_bits == 64, "dlrm_qr_expand_csr: bad offset_bits");
  const int64_t per = max_lookups_per_table > B ? max_lookups_per_table : B;
  int64_t bx = dlrm::ceil_div(per, 256);
  if (bx > 4096) bx = 4096;  // grid-stride beyond
  const dim3 grid((unsigned)bx, (unsigned)T_phys), block(256);
  hipStream_t st = dlrm::as_stream(stream);
#define QX(I, O)                                                                              \
  hipLaunchKernelGGL((qr_expand_kernel<I, O>), grid, block, 0, st, T_phys, B,                  \
                     static_cast<const I*>(indices), static_cast<const O*>(offsets), src, kind, \
                     coll, phys_indices, phys_offsets, phys_capacity, error_flag)
  if (index_bits == 32 && offset_bits == 32) QX(int32_t, int32_t);
  else if (index_bits == 32) QX(int32_t, int64_t);
  else if (offset_bits == 32) QX(int64_t, int32_t);
  else QX(int64_t, int64_t);
#undef QX
  DLRM_LAUNCH_CHECK("dlrm_qr_expand_csr");
  return DLRM_OK;
}

extern "C" int dlrm_qr_pool_combine_forward(int32_t op, int32_t T, int64_t B, int64_t D,
                                            const int32_t* pq, const int32_t* pr, const float* P,
                                            int64_t p_batch_stride, float* E,
                                            int64_t e_batch_stride, dlrm_stream_t stream) {
  DLRM_ARG(op == DLRM_QR_MULT || op == DLRM_QR_ADD, "dlrm_qr_pool_combine_forward: mult or add");
  DLRM_ARG(T > 0 && B >= 0 && D > 0 && D % 4 == 0 && p_batch_stride % 4 == 0 &&
               e_batch_stride % 4 == 0,
           "dlrm_qr_pool_combine_forward: bad sizes (D and strides multiples of 4)");
  if (B == 0) return DLRM_OK;
  DLRM_ARG(pq && pr && P && E, "dlrm_qr_pool_combine_forward: null pointer");
  const int64_t n = B * T * (D / 4);
  hipLaunchKernelGGL(qr_pool_fwd_kernel, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), op, T, B, D / 4, pq, pr,
                     reinterpret_cast<const float4*>(P), p_batch_stride / 4,
                     reinterpret_cast<float4*>(E), e_batch_stride / 4);
  DLRM_LAUNCH_CHECK("dlrm_qr_pool_combine_forward");
  return DLRM_OK;
}

extern "C" int dlrm_qr_pool_combine_backward(int32_t op, int32_t T, int64_t B, int64_t D,
                                             const int32_t* pq, const int32_t* pr, const float* P,
                                             int64_t p_batch_stride, const float* dE,
                                             int64_t e_batch_stride, float* dP,
                                             int64_t dp_batch_stride, dlrm_stream_t stream) {
  DLRM_ARG(op == DLRM_QR_MULT || op == DLRM_QR_ADD, "dlrm_qr_pool_combine_backward: mult or add");
  DLRM_ARG(T > 0 && B >= 0 && D > 0 && D % 4 == 0 && p_batch_stride % 4 == 0 &&
               e_batch_stride % 4 == 0 && dp_batch_stride % 4 == 0,
           "dlrm_qr_pool_combine_backward: bad sizes (D and strides multiples of 4)");
  if (B == 0) return DLRM_OK;
  DLRM_ARG(pq && pr && P && dE && dP, "dlrm_qr_pool_combine_backward: null pointer");
  const int64_t n = B * T * (D / 4);
  hipLaunchKernelGGL(qr_pool_bwd_kernel, dim3(dlrm::ceil_div(n, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), op, T, B, D / 4, pq, pr,
                     reinterpret_cast<const float4*>(P), p_batch_stride / 4,
                     reinterpret_cast<const float4*>(dE), e_batch_stride / 4,
                     reinterpret_cast<float4*>(dP), dp_batch_stride / 4);
  DLRM_LAUNCH_CHECK("dlrm_qr_pool_combine_backward");
  return DLRM_OK;
}

extern "C" int dlrm_qr_split_indices(const void* indices, int32_t index_bits, int64_t n,
                                     int64_t collisions, int64_t* q_out, int64_t* r_out,
                                     dlrm_stream_t stream) {
  DLRM_ARG(n == 0 || (indices && q_out && r_out), "dlrm_qr_split_indices: null pointer");
  DLRM_ARG(collisions > 0, "dlrm_qr_split_indices: collisions must be > 0");
  DLRM_ARG(index_bits == 32 || index_bits == 64, "dlrm_qr_split_indices: bad index_bits");
  if (n == 0) return DLRM_OK;
  hipStream_t st = dlrm::as_stream(stream);
  const int64_t blocks = dlrm::ceil_div(n, 256);
  if (index_bits == 32)
    hipLaunchKernelGGL(qr_split_kernel<int32_t>, dim3(blocks), dim3(256), 0, st,
                       static_cast<const int32_t*>(indices), n, collisions, q_out, r_out);
  else
    hipLaunchKernelGGL(qr_split_kernel<int64_t>, dim3(blocks), dim3(256), 0, st,
                       static_cast<const int64_t*>(indices), n, collisions, q_out, r_out);
  DLRM_LAUNCH_CHECK("dlrm_qr_split_indices");
  return DLRM_OK;
}

extern "C" int dlrm_qr_combine_forward(int32_t op, int64_t n_rows, int64_t D, const float* eq,
                                       const float* er, float* out, dlrm_stream_t stream) {
  DLRM_ARG(op >= 0 && op <= 2, "dlrm_qr_combine_forward: bad op");
  DLRM_ARG(n_rows >= 0 && D > 0, "dlrm_qr_combine_forward: bad sizes");
  if (n_rows == 0) return DLRM_OK;
  DLRM_ARG(eq && er && out, "dlrm_qr_combine_forward: null pointer");
  hipLaunchKernelGGL(qr_combine_fwd_kernel, dim3(dlrm::ceil_div(n_rows * D, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), op, n_rows, D, eq, er, out);
  DLRM_LAUNCH_CHECK("dlrm_qr_combine_forward");
  return DLRM_OK;
}

extern "C" int dlrm_qr_combine_backward(int32_t op, int64_t n_rows, int64_t D, const float* eq,
                                        const float* er, const float* grad_out, float* grad_eq,
                                        float* grad_er, dlrm_stream_t stream) {
  DLRM_ARG(op >= 0 && op <= 2, "dlrm_qr_combine_backward: bad op");
  DLRM_ARG(n_rows >= 0 && D > 0, "dlrm_qr_combine_backward: bad sizes");
  if (n_rows == 0) return DLRM_OK;
  DLRM_ARG(eq && er && grad_out && grad_eq && grad_er, "dlrm_qr_combine_backward: null pointer");
  hipLaunchKernelGGL(qr_combine_bwd_kernel, dim3(dlrm::ceil_div(n_rows * D, 256)), dim3(256), 0,
                     dlrm::as_stream(stream), op, n_rows, D, eq, er, grad_out, grad_eq, grad_er);
  DLRM_LAUNCH_CHECK("dlrm_qr_combine_backward");
  return DLRM_OK;
}

extern "C" int dlrm_csr_from_tables(int32_t T, int32_t B, const int64_t* const* table_offsets,
                                    const int64_t* table_nnz, void* out_offsets,
                                    int32_t out_offset_bits, dlrm_stream_t stream) {
  DLRM_ARG(T > 0 && T <= 64 && B > 0, "dlrm_csr_from_tables: need 0 < T <= 64, B > 0");
  DLRM_ARG(table_offsets && table_nnz && out_offsets, "dlrm_csr_from_tables: null pointer");
  DLRM_ARG(out_offset_bits == 32 || out_offset_bits == 64, "dlrm_csr_from_tables: bad bits");
  CsrArgs a{};
  a.start[0] = 0;
  for (int t = 0; t < T; ++t) {
    DLRM_ARG(table_offsets[t] != nullptr, "dlrm_csr_from_tables: null table offsets");
    a.off[t] = table_offsets[t];
    a.start[t + 1] = a.start[t] + table_nnz[t];
  }
  const int64_t n = (int64_t)T * B + 1;
  hipStream_t st = dlrm::as_stream(stream);
  if (out_offset_bits == 32) {
    DLRM_REQUIRE(a.start[T] < (int64_t)INT32_MAX, DLRM_ERR_UNSUPPORTED,
                 "dlrm_csr_from_tables: int32 offsets overflow");
    hipLaunchKernelGGL(csr_from_tables_kernel<int32_t>, dim3(dlrm::ceil_div(n, 256)), dim3(256),
                       0, st, T, B, a, static_cast<int32_t*>(out_offsets));
  } else {
    hipLaunchKernelGGL(csr_from_tables_kernel<int64_t>, dim3(dlrm::ceil_div(n, 256)), dim3(256),
                       0, st, T, B, a, static_cast<int64_t*>(out_offsets));
  }
  DLRM_LAUNCH_CHECK("dlrm_csr_from_tables");
  return DLRM_OK;
}

extern "C" int dlrm_tbe_expand_grad(int64_t D, int32_t T, int32_t B, const void* offsets,
                                    int32_t offset_bits, int64_t num_lookups,
                                    const float* per_sample_weights, const float* grad_out,
                                    int64_t grad_batch_stride, float* values,
                                    dlrm_stream_t stream) {
  const char* name = "dlrm_tbe_expand_grad";
  DLRM_ARG(D > 0 && T > 0 && B > 0 && num_lookups >= 0, "%s: bad sizes", name);
  if (num_lookups == 0) return DLRM_OK;
  DLRM_ARG(offsets && grad_out && values, "%s: null pointer", name);
  DLRM_ARG(offset_bits == 32 || offset_bits == 64, "%s: bad offset_bits", name);
  DLRM_ARG(grad_batch_stride >= (int64_t)T * D, "%s: grad_batch_stride < T*D", name);
  int64_t blocks = dlrm::ceil_div(num_lookups, 4);
  if (blocks > 16384) blocks = 16384;
  hipStream_t st = dlrm::as_stream(stream);
  if (offset_bits == 32)
    hipLaunchKernelGGL(tbe_expand_grad_kernel<int32_t>, dim3(blocks), dim3(256), 0, st, D, T, B,
                       static_cast<const int32_t*>(offsets), num_lookups, per_sample_weights,
                       grad_out, grad_batch_stride, values);
  else
    hipLaunchKernelGGL(tbe_expand_grad_kernel<int64_t>, dim3(blocks), dim3(256), 0, st, D, T, B,
                       static_cast<const int64_t*>(offsets), num_lookups, per_sample_weights,
                       grad_out, grad_batch_stride, values);
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}

extern "C" int dlrm_tbe_psw_grad(const float* weights, int64_t D, const int64_t* row_base,
                                 int32_t T, int32_t B, const void* indices, int32_t index_bits,
                                 const void* offsets, int32_t offset_bits, int64_t num_lookups,
                                 const float* grad_out, int64_t grad_batch_stride,
                                 float* grad_per_sample_weights, dlrm_stream_t stream) {
  const char* name = "dlrm_tbe_psw_grad";
  DLRM_ARG(D > 0 && T > 0 && B > 0 && num_lookups >= 0, "%s: bad sizes", name);
  if (num_lookups == 0) return DLRM_OK;
  DLRM_ARG(weights && row_base && indices && offsets && grad_out && grad_per_sample_weights,
           "%s: null pointer", name);
  DLRM_ARG(index_bits == 32 || index_bits == 64, "%s: bad index_bits", name);
  DLRM_ARG(offset_bits == 32 || offset_bits == 64, "%s: bad offset_bits", name);
  DLRM_ARG(grad_batch_stride >= (int64_t)T * D, "%s: grad_batch_stride < T*D", name);
  int64_t blocks = dlrm::ceil_div(num_lookups, 4);
  if (blocks > 16384) blocks = 16384;
  hipStream_t st = dlrm::as_stream(stream);
#define PG(I, O)                                                                             \
  hipLaunchKernelGGL((tbe_psw_grad_kernel<I, O>), dim3(blocks), dim3(256), 0, st, weights, D, \
                     row_base, T, B, static_cast<const I*>(indices),                          \
                     static_cast<const O*>(offsets), num_lookups, grad_out, grad_batch_stride, \
                     grad_per_sample_weights)
  if (index_bits == 32 && offset_bits == 32) PG(int32_t, int32_t);
  else if (index_bits == 32) PG(int32_t, int64_t);
  else if (offset_bits == 32) PG(int64_t, int32_t);
  else PG(int64_t, int64_t);
#undef PG
  DLRM_LAUNCH_CHECK(name);
  return DLRM_OK;
}
