// Tensor glue for the batched bwd-data weight preparation (kernels/wprep.hip): the job table is
// built once per set of registered convolutions (ops/wprep.py) and stays on the device; each step
// runs one launch over it.
#include <ATen/ATen.h>

#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <cstring>
#include <tuple>
#include <vector>

#include "kernels/launchers_wprep.h"
#include "ops.h"

namespace psd {

// geo: 6 ints per job (Rp, Sp, r0, s0, sr, ss). Returns (device table, total tiles).
std::tuple<at::Tensor, int64_t> wprep_table(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts,
                                            const std::vector<int64_t>& geo) {
  const size_t J = srcs.size();
  TORCH_CHECK(J > 0 && dsts.size() == J && geo.size() == 6 * J, "psd wprep: srcs / dsts / geo (6 per job) mismatch");
  std::vector<WprepJob> jobs(J);
  int64_t tiles = 0;
  for (size_t i = 0; i < J; ++i) {
    const at::Tensor& s = srcs[i];
    const at::Tensor& d = dsts[i];
    TORCH_CHECK(s.is_cuda() && s.scalar_type() == at::kBFloat16 && s.dim() == 4 &&
                    s.is_contiguous(at::MemoryFormat::ChannelsLast),
                "psd wprep: src must be a channels_last bf16 [co, ci, R, S] weight");
    const int co = s.size(0), ci = s.size(1), R = s.size(2), S = s.size(3);
    const int Rp = geo[6 * i], Sp = geo[6 * i + 1], r0 = geo[6 * i + 2], s0 = geo[6 * i + 3];
    const int sr = geo[6 * i + 4], ss = geo[6 * i + 5];
    TORCH_CHECK(co % 8 == 0 && ci % 8 == 0, "psd wprep: co and ci must be multiples of 8");
    TORCH_CHECK(Rp >= 1 && Sp >= 1 && r0 >= 0 && r0 < R && s0 >= 0 && s0 < S && r0 + (Rp - 1) * sr >= 0 &&
                    r0 + (Rp - 1) * sr < R && s0 + (Sp - 1) * ss >= 0 && s0 + (Sp - 1) * ss < S,
                "psd wprep: tap subset outside the kernel window");
    TORCH_CHECK(d.is_cuda() && d.scalar_type() == at::kBFloat16 && d.is_contiguous() &&
                    d.numel() == (int64_t)ci * Rp * Sp * co && d.device() == s.device() &&
                    (reinterpret_cast<uintptr_t>(d.data_ptr()) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(s.data_ptr()) & 15) == 0,
                "psd wprep: dst must be a contiguous 16-B aligned bf16 [ci, Rp * Sp * co] on the src's device");
    WprepJob& j = jobs[i];
    j.src = reinterpret_cast<const uint16_t*>(s.data_ptr());
    j.dst = reinterpret_cast<uint16_t*>(d.data_ptr());
    j.co = co; j.ci = ci; j.R = R; j.S = S; j.Rp = Rp; j.Sp = Sp;
    j.r0 = r0; j.s0 = s0; j.sr = sr; j.ss = ss;
    j.tile0 = (int)tiles;
    j.pad_ = 0;
    tiles += wprep_tiles(co, ci, Rp, Sp);
    TORCH_CHECK(tiles < (1LL << 31), "psd wprep: too many tiles");
  }
  at::Tensor host = at::empty({(int64_t)(J * sizeof(WprepJob))}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), jobs.data(), J * sizeof(WprepJob));
  return {host.to(srcs[0].device()), tiles};
}

void wprep_run(const at::Tensor& table, int64_t tiles) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kByte && table.numel() % sizeof(WprepJob) == 0,
              "psd wprep: table must come from wprep_table");
  const c10::DeviceGuard g(table.device());
  const int njobs = (int)(table.numel() / sizeof(WprepJob));
  hipError_t e = launch_wprep(reinterpret_cast<const WprepJob*>(table.data_ptr()), njobs, (int)tiles,
                              c10::hip::getCurrentHIPStream(table.device().index()).stream());
  TORCH_CHECK(e == hipSuccess, "psd wprep: ", hipGetErrorString(e));
}

}  // namespace psd
