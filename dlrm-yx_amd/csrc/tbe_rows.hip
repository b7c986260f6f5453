// Table-batched EmbeddingBag forward over reduced-precision rows:
//   DLRM_ROWS_F16 : fp16 weights, the fbgemm TBE's weights_precision=FP16 tables
//                   (DLRM_Net.create_emb_fbgemm, dlrm_s_pytorch.py:337-366);
//   DLRM_ROWS_Q8  : 8-bit row-wise quantized rows as packed by
//                   torch.ops.quantized.embedding_bag_byte_prepack (D uint8, then fp32
//                   scale, fp32 bias), looked up by embedding_bag_byte_rowwise_offsets
//                   (DLRM_Net.quantize_embedding / apply_emb, :554-567, 609-625);
//   DLRM_ROWS_Q4  : 4-bit row-wise (embedding_bag_4bit_prepack: ceil(D/2) bytes, element
//                   2i in the low nibble of byte i, then fp16 scale, fp16 bias).
// Dequantised value = q * scale + bias; a bag's sum accumulates in fp32 as
// acc = fma(w*scale, q, acc + w*bias) (w = per-sample weight or 1).
//
// Same data layout and launch shape as the fp32 lookup (tbe.hip): all tables in one
// buffer of fixed-size rows, table t = rows [row_base[t], row_base[t+1]), one group of LPB
// lanes per (table, bag), every lane owning 4 consecutive elements per 4*LPB, four rows of
// a bag in flight.  HBM-bound: a C3 row is 512 B in fp32, 256 B in fp16, 136 B in Q8 and
// 68 B in Q4, so the gather moves 2x / 3.8x / 7.5x fewer bytes.
#include "common.hpp"

namespace {

using dlrm::kWave;

__device__ __forceinline__ float half_bits_to_float(uint32_t h) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)h);
}

// Decode elements 4c .. 4c+3 of a row (quantized: the raw levels q).
template <int FMT>
__device__ __forceinline__ float4 load4(const uint8_t* __restrict__ row, int c) {
  if constexpr (FMT == DLRM_ROWS_F16) {
    const uint2 u = *reinterpret_cast<const uint2*>(row + 8 * c);
    return make_float4(half_bits_to_float(u.x & 0xffff), half_bits_to_float(u.x >> 16),
                       half_bits_to_float(u.y & 0xffff), half_bits_to_float(u.y >> 16));
  } else if constexpr (FMT == DLRM_ROWS_Q8) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(row + 4 * c);
    return make_float4((float)(u & 0xff), (float)((u >> 8) & 0xff), (float)((u >> 16) & 0xff),
                       (float)(u >> 24));
  } else {
    const uint32_t u = *reinterpret_cast<const uint16_t*>(row + 2 * c);
    return make_float4((float)(u & 0xf), (float)((u >> 4) & 0xf), (float)((u >> 8) & 0xf),
                       (float)((u >> 12) & 0xf));
  }
}

template <int FMT>
__device__ __forceinline__ float2 scale_bias(const uint8_t* __restrict__ row, int64_t D) {
  if constexpr (FMT == DLRM_ROWS_Q8) {  // rows are 4-byte aligned (D % 4 == 0)
    const float* sb = reinterpret_cast<const float*>(row + D);
    return make_float2(sb[0], sb[1]);
  } else if constexpr (FMT == DLRM_ROWS_Q4) {  // rows are 2-byte aligned
    const uint16_t* sb = reinterpret_cast<const uint16_t*>(row + (D + 1) / 2);
    return make_float2(half_bits_to_float(sb[0]), half_bits_to_float(sb[1]));
  } else {
    return make_float2(1.f, 0.f);
  }
}

template <int FMT, int LPB, int MAXV, typename IdxT, typename OffT>
__global__ __launch_bounds__(256) void tbe_rows_fwd_kernel(
    const uint8_t* __restrict__ Wb, int64_t row_bytes, int64_t D,
    const int64_t* __restrict__ row_base, int T, int B, const IdxT* __restrict__ idx,
    const OffT* __restrict__ off, const float* __restrict__ psw, float* __restrict__ out,
    int64_t out_bs, int32_t* __restrict__ err) {
  constexpr int GPW = kWave / LPB;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPB;
  const int gl = lane - g * LPB;
  const int nchunks = (int)(D / 4);
  const int64_t nbags = (int64_t)T * B;
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / kWave);

  for (int64_t bag0 = wave_id * GPW; bag0 < nbags; bag0 += nwaves * GPW) {
    const int64_t bag = bag0 + g;
    const bool active = bag < nbags;
    int t = 0, b = 0;
    int64_t start = 0, end = 0, base = 0, nrows = 0;
    if (active) {
      t = (int)(bag / B);
      b = (int)(bag - (int64_t)t * B);
      start = (int64_t)off[bag];
      end = (int64_t)off[bag + 1];
      base = row_base[t];
      nrows = row_base[t + 1] - base;
    }
    float4 acc[MAXV];
#pragma unroll
    for (int c = 0; c < MAXV; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);

    for (int64_t l0 = start; l0 < end; l0 += LPB) {
      const int n = (int)((end - l0) < LPB ? (end - l0) : LPB);
      int64_t my_row = -1;
      float my_w = 1.f;
      if (gl < n) {
        int64_t r = (int64_t)idx[l0 + gl];
        if (r < 0 || r >= nrows) {
          if (err) atomicOr(err, DLRM_TBE_ERR_INDEX);
          r = -1;
        }
        my_row = r;
        if (psw) my_w = psw[l0 + gl];
      }
      for (int j = 0; j < n; j += 4) {
        int64_t r[4];
        float w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int src = g * LPB + ((j + u) < LPB ? (j + u) : 0);
          r[u] = __shfl(my_row, src, kWave);
          w[u] = __shfl(my_w, src, kWave);
          if (j + u >= n) r[u] = -1;
        }
        // all four rows' loads issued before any is used (invalid rows read row 0 of the
        // table and are dropped at the accumulation)
        float4 v[4][MAXV];
        float2 sb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint8_t* row = Wb + (base + (r[u] >= 0 ? r[u] : 0)) * row_bytes;
          sb[u] = scale_bias<FMT>(row, D);
#pragma unroll
          for (int c = 0; c < MAXV; ++c) {
            const int chunk = gl + c * LPB;
            v[u][c] = load4<FMT>(row, chunk < nchunks ? chunk : 0);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (r[u] >= 0) {
            const float ws = w[u] * sb[u].x, wb = w[u] * sb[u].y;
#pragma unroll
            for (int c = 0; c < MAXV; ++c) {
              if (FMT == DLRM_ROWS_F16) {
                acc[c].x = fmaf(w[u], v[u][c].x, acc[c].x);
                acc[c].y = fmaf(w[u], v[u][c].y, acc[c].y);
                acc[c].z = fmaf(w[u], v[u][c].z, acc[c].z);
                acc[c].w = fmaf(w[u], v[u][c].w, acc[c].w);
              } else {
                acc[c].x = fmaf(ws, v[u][c].x, acc[c].x + wb);
                acc[c].y = fmaf(ws, v[u][c].y, acc[c].y + wb);
                acc[c].z = fmaf(ws, v[u][c].z, acc[c].z + wb);
                acc[c].w = fmaf(ws, v[u][c].w, acc[c].w + wb);
              }
            }
          }
        }
      }
    }
    if (active) {
      float4* o = reinterpret_cast<float4*>(out + (int64_t)b * out_bs + (int64_t)t * D);
#pragma unroll
      for (int c = 0; c < MAXV; ++c) {
        const int chunk = gl + c * LPB;
        if (chunk < nchunks) o[chunk] = acc[c];
      }
    }
  }
}

int64_t min_row_bytes(int fmt, int64_t D) {
  switch (fmt) {
    case DLRM_ROWS_F16: return 2 * D;
    case DLRM_ROWS_Q8: return D + 8;
    case DLRM_ROWS_Q4: return (D + 1) / 2 + 4;
    default: return -1;
  }
}

template <int FMT, typename IdxT, typename OffT>
int launch_rows_fwd(const uint8_t* W, int64_t row_bytes, int64_t D, const int64_t* row_base,
                    int T, int B, const void* idx, const void* off, const float* psw, float* out,
                    int64_t out_bs, int32_t* err, hipStream_t st) {
  const int64_t nchunks = D / 4;
  int lpb = 4;
  while (lpb < nchunks && lpb < 64) lpb <<= 1;
  const int64_t maxv = dlrm::ceil_div(nchunks, lpb);
  const int64_t nbags = (int64_t)T * B;
  const int gpw = 64 / lpb;
  int64_t blocks = dlrm::ceil_div(dlrm::ceil_div(nbags, gpw), 4);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  const IdxT* ip = static_cast<const IdxT*>(idx);
  const OffT* op = static_cast<const OffT*>(off);
#define RF(LPB, MV)                                                                         \
  hipLaunchKernelGGL((tbe_rows_fwd_kernel<FMT, LPB, MV, IdxT, OffT>), dim3(blocks), dim3(256), \
                     0, st, W, row_bytes, D, row_base, T, B, ip, op, psw, out, out_bs, err)
  switch (lpb) {
    case 4: RF(4, 1); break;
    case 8: RF(8, 1); break;
    case 16: RF(16, 1); break;
    case 32: RF(32, 1); break;
    default:
      if (maxv == 1)
        RF(64, 1);
      else
        RF(64, 2);
  }
#undef RF
  DLRM_LAUNCH_CHECK("dlrm_tbe_forward_rows");
  return DLRM_OK;
}

template <int FMT>
int rows_dispatch(const uint8_t* W, int64_t row_bytes, int64_t D, const int64_t* row_base, int T,
                  int B, const void* idx, int ib, const void* off, int ob, const float* psw,
                  float* out, int64_t out_bs, int32_t* err, hipStream_t st) {
  if (ib == 32 && ob == 32)
    return launch_rows_fwd<FMT, int32_t, int32_t>(W, row_bytes, D, row_base, T, B, idx, off, psw,
                                                  out, out_bs, err, st);
  if (ib == 32)
    return launch_rows_fwd<FMT, int32_t, int64_t>(W, row_bytes, D, row_base, T, B, idx, off, psw,
                                                  out, out_bs, err, st);
  if (ob == 32)
    return launch_rows_fwd<FMT, int64_t, int32_t>(W, row_bytes, D, row_base, T, B, idx, off, psw,
                                                  out, out_bs, err, st);
  return launch_rows_fwd<FMT, int64_t, int64_t>(W, row_bytes, D, row_base, T, B, idx, off, psw,
                                                out, out_bs, err, st);
}

}  // namespace

extern "C" int64_t dlrm_tbe_row_bytes(int32_t format, int64_t D) { return min_row_bytes(format, D); }

extern "C" int dlrm_tbe_forward_rows(const void* weights, int32_t format, int64_t row_bytes,
                                     int64_t D, const int64_t* row_base, int32_t T, int32_t B,
                                     const void* indices, int32_t index_bits, const void* offsets,
                                     int32_t offset_bits, const float* per_sample_weights,
                                     float* out, int64_t out_batch_stride, int32_t* error_flag,
                                     dlrm_stream_t stream) {
  const char* name = "dlrm_tbe_forward_rows";
  DLRM_ARG(weights && row_base && out && offsets && indices, "%s: null pointer", name);
  DLRM_ARG(format == DLRM_ROWS_F16 || format == DLRM_ROWS_Q8 || format == DLRM_ROWS_Q4,
           "%s: bad row format %d", name, format);
  DLRM_ARG(T >= 0 && B >= 0 && D > 0, "%s: bad sizes", name);
  DLRM_ARG(index_bits == 32 || index_bits == 64, "%s: index_bits must be 32|64", name);
  DLRM_ARG(offset_bits == 32 || offset_bits == 64, "%s: offset_bits must be 32|64", name);
  DLRM_ARG(row_bytes >= min_row_bytes(format, D), "%s: row_bytes %lld < %lld", name,
           (long long)row_bytes, (long long)min_row_bytes(format, D));
  DLRM_ARG(out_batch_stride >= (int64_t)T * D, "%s: out_batch_stride < T*D", name);
  DLRM_REQUIRE(D % 4 == 0 && D <= 512, DLRM_ERR_UNSUPPORTED,
               "%s: D must be a multiple of 4 and <= 512 (D=%lld)", name, (long long)D);
  const int align = format == DLRM_ROWS_F16 ? 8 : (format == DLRM_ROWS_Q8 ? 4 : 2);
  DLRM_REQUIRE((reinterpret_cast<uintptr_t>(weights) % align) == 0 && row_bytes % align == 0 &&
                   (reinterpret_cast<uintptr_t>(out) & 15) == 0 && out_batch_stride % 4 == 0,
               DLRM_ERR_UNSUPPORTED, "%s: misaligned rows or output", name);
  if ((int64_t)T * B == 0) return DLRM_OK;
  hipStream_t st = dlrm::as_stream(stream);
  const uint8_t* W = static_cast<const uint8_t*>(weights);
  switch (format) {
    case DLRM_ROWS_F16:
      return rows_dispatch<DLRM_ROWS_F16>(W, row_bytes, D, row_base, T, B, indices, index_bits,
                                          offsets, offset_bits, per_sample_weights, out,
                                          out_batch_stride, error_flag, st);
    case DLRM_ROWS_Q8:
      return rows_dispatch<DLRM_ROWS_Q8>(W, row_bytes, D, row_base, T, B, indices, index_bits,
                                         offsets, offset_bits, per_sample_weights, out,
                                         out_batch_stride, error_flag, st);
    default:
      return rows_dispatch<DLRM_ROWS_Q4>(W, row_bytes, D, row_base, T, B, indices, index_bits,
                                         offsets, offset_bits, per_sample_weights, out,
                                         out_batch_stride, error_flag, st);
  }
}
