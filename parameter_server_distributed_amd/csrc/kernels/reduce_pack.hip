// Multi-source gradient reduce and many-tensor pack/cast for gfx950.
//
// multi_reduce: out = scale * sum_k src_k. Replaces the reference's per-(tensor, worker, element)
// host loop (src/parameter_server.cpp:38-63) for gradients that arrive as K separate inboxes
// (p2p pushes to a PS shard that is not colocated with the workers, or async pushes batched by
// the apply thread). Streaming, 8 elements/lane, 16-byte loads.
//
// pack_cast: gathers many small tensors into one flat bucket (or scatters back) with an
// fp32<->bf16 cast, one launch for the whole model. Replaces the per-element proto encode/decode
// (src/worker.cpp:40-66, src/parameter_server_service.cpp:35-42,70-80) on the bulk-tensor path.
#include "common.h"
#include "launchers.h"

namespace psd {

template <int SRC_DT, int OUT_DT>
__global__ __launch_bounds__(256) void multi_reduce_kernel(SourceList s, void* __restrict__ out, float scale,
                                                           int64_t n) {
  const int64_t nvec = n >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t i = v << 3;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int k = 0; k < s.count; ++k) {
      float t[8];
      if (SRC_DT == DT_BF16)
        load8_bf16(static_cast<const uint16_t*>(s.ptr[k]) + i, t);
      else
        load8_f32(static_cast<const float*>(s.ptr[k]) + i, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += t[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= scale;
    if (OUT_DT == DT_BF16)
      store8_bf16(static_cast<uint16_t*>(out) + i, acc);
    else
      store8_f32(static_cast<float*>(out) + i, acc);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      float acc = 0.f;
      for (int k = 0; k < s.count; ++k)
        acc += (SRC_DT == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(s.ptr[k])[i])
                                   : static_cast<const float*>(s.ptr[k])[i];
      acc *= scale;
      if (OUT_DT == DT_BF16)
        static_cast<uint16_t*>(out)[i] = f32_to_bf16(acc);
      else
        static_cast<float*>(out)[i] = acc;
    }
  }
}

hipError_t launch_multi_reduce(const SourceList& s, void* out, int32_t out_dtype, float scale, int64_t n,
                               hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (s.count < 1 || s.count > kMaxSources) return hipErrorInvalidValue;
  const int block = 256;
  const int grid = stream_grid((n >> 3) > 0 ? (n >> 3) : 1, block);
#define PSD_RED(SD, OD) \
  hipLaunchKernelGGL((multi_reduce_kernel<SD, OD>), dim3(grid), dim3(block), 0, st, s, out, scale, n)
  if (s.dtype == DT_BF16 && out_dtype == DT_BF16) PSD_RED(DT_BF16, DT_BF16);
  else if (s.dtype == DT_BF16 && out_dtype == DT_F32) PSD_RED(DT_BF16, DT_F32);
  else if (s.dtype == DT_F32 && out_dtype == DT_BF16) PSD_RED(DT_F32, DT_BF16);
  else if (s.dtype == DT_F32 && out_dtype == DT_F32) PSD_RED(DT_F32, DT_F32);
  else return hipErrorInvalidValue;
#undef PSD_RED
  return hipGetLastError();
}

constexpr int64_t kPackChunk = 8192;

template <int SD, int DD>
__device__ __forceinline__ void cast_store(const void* src, void* dst, int64_t i) {
  float x = (SD == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(src)[i]) : static_cast<const float*>(src)[i];
  if (DD == DT_BF16)
    static_cast<uint16_t*>(dst)[i] = f32_to_bf16(x);
  else
    static_cast<float*>(dst)[i] = x;
}

// One block per 8K-element chunk of one segment. Vector path when the segment is 16-B aligned
// on both sides and its chunk is a whole number of 8-element groups (the common case: the
// runtime pads every tensor to 8 elements inside its flat buckets); scalar otherwise.
template <int SD, int DD>
__global__ __launch_bounds__(256) void pack_cast_kernel(const PackSeg* __restrict__ segs,
                                                        const int32_t* __restrict__ chunk_seg,
                                                        const int64_t* __restrict__ chunk_off) {
  const PackSeg sg = segs[chunk_seg[blockIdx.x]];
  const int64_t beg = chunk_off[blockIdx.x];
  const int64_t end = min(beg + kPackChunk, sg.numel);
  const bool aligned = ((((uintptr_t)sg.src) | ((uintptr_t)sg.dst)) & 15u) == 0;
  if (aligned) {
    const int64_t vend = beg + ((end - beg) & ~(int64_t)7);
    for (int64_t i = beg + (int64_t)threadIdx.x * 8; i < vend; i += (int64_t)blockDim.x * 8) {
      float t[8];
      if (SD == DT_BF16) load8_bf16(static_cast<const uint16_t*>(sg.src) + i, t);
      else load8_f32(static_cast<const float*>(sg.src) + i, t);
      if (DD == DT_BF16) store8_bf16(static_cast<uint16_t*>(sg.dst) + i, t);
      else store8_f32(static_cast<float*>(sg.dst) + i, t);
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += blockDim.x) cast_store<SD, DD>(sg.src, sg.dst, i);
  } else {
    for (int64_t i = beg + threadIdx.x; i < end; i += blockDim.x) cast_store<SD, DD>(sg.src, sg.dst, i);
  }
}

hipError_t launch_pack_cast(const PackSeg* segs, const int32_t* chunk_seg, const int64_t* chunk_off,
                            int64_t n_chunks, int32_t sd, int32_t dd, hipStream_t st) {
  if (n_chunks <= 0) return hipSuccess;
#define PSD_PACK(S, D) \
  hipLaunchKernelGGL((pack_cast_kernel<S, D>), dim3((unsigned)n_chunks), dim3(256), 0, st, segs, chunk_seg, chunk_off)
  if (sd == DT_F32 && dd == DT_F32) PSD_PACK(DT_F32, DT_F32);
  else if (sd == DT_F32 && dd == DT_BF16) PSD_PACK(DT_F32, DT_BF16);
  else if (sd == DT_BF16 && dd == DT_F32) PSD_PACK(DT_BF16, DT_F32);
  else if (sd == DT_BF16 && dd == DT_BF16) PSD_PACK(DT_BF16, DT_BF16);
  else return hipErrorInvalidValue;
#undef PSD_PACK
  return hipGetLastError();
}

}  // namespace psd
