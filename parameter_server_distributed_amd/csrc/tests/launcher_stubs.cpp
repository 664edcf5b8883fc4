// Host-only sanitizer builds of the PS cores: the gfx950 launchers referenced by ops.cpp, as stubs
// (only CPU tensors reach ops.cpp in those builds; a device call fails loudly instead of linking HIP
// device code into a TSAN/ASAN binary).
#include "../kernels/launchers.h"
#include "../kernels/launchers_xfer.h"

namespace psd {
hipError_t launch_fused_apply(const OptimHyper&, const OptimDyn*, float*, const SourceList&, float*, float*, uint16_t*,
                              int64_t, hipStream_t, int) {
  return hipErrorNotSupported;
}
hipError_t launch_optim_advance(OptimDyn*, float, float, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_multi_reduce(const SourceList&, void*, int32_t, float, int64_t, hipStream_t) {
  return hipErrorNotSupported;
}
hipError_t launch_pack_cast(const PackSeg*, const int32_t*, const int64_t*, int64_t, int32_t, int32_t, hipStream_t) {
  return hipErrorNotSupported;
}
hipError_t launch_amax(const void*, int32_t, int64_t, float*, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_quant_fp8(const void*, int32_t, int64_t, const float*, float, uint8_t*, float*, hipStream_t, int) {
  return hipErrorNotSupported;
}
hipError_t launch_quant_fp8_jit(const void*, int32_t, int64_t, float*, float, uint8_t*, float*, hipStream_t, int) {
  return hipErrorNotSupported;
}
hipError_t launch_quant_fp8_delayed(const void*, int32_t, int64_t, float*, float, float, uint8_t*, float*, hipStream_t,
                                    int) {
  return hipErrorNotSupported;
}
hipError_t launch_dequant_fp8(const uint8_t*, int64_t, const float*, void*, int32_t, hipStream_t) {
  return hipErrorNotSupported;
}
hipError_t launch_quant_mx(const void*, int32_t, int64_t, int, uint8_t*, uint8_t*, hipStream_t) {
  return hipErrorNotSupported;
}
hipError_t launch_dequant_mx(const uint8_t*, const uint8_t*, int64_t, void*, int32_t, hipStream_t) {
  return hipErrorNotSupported;
}
hipError_t launch_xfer(const XferList&, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_xfer_mx(const XferMxList&, hipStream_t) { return hipErrorNotSupported; }
}  // namespace psd
