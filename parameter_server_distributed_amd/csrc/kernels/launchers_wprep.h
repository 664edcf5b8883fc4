// Launch API of the batched bwd-data weight preparation (wprep.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {

// one output operand: dst[ci][r'][s'][co] = src[co][r0 + r' sr][s0 + s' ss][ci] (bf16; src the OHWI /
// channels_last storage of a [co, ci, R, S] weight; co, ci multiples of 8)
struct WprepJob {
  const uint16_t* src;
  uint16_t* dst;
  int co, ci, R, S, Rp, Sp, r0, s0, sr, ss;
  int tile0;  // first block of this job (ascending over the table)
  int pad_;
};

// blocks one job takes
int wprep_tiles(int co, int ci, int Rp, int Sp);
// jobs_dev: a device-resident table of njobs jobs whose tiles cover [0, total_tiles)
hipError_t launch_wprep(const WprepJob* jobs_dev, int njobs, int total_tiles, hipStream_t stream);

}  // namespace psd
