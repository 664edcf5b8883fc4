// Checkpoint I/O.
//
// 1. Reference format, bit-exact (src/parameter_server.cpp:112-188): native-endian
//      int32 epoch | int32 iteration | u64 n |
//      n x { u64 name_len | name | u64 rank | int32[rank] shape | int32 dtype | u64 numel | f32[numel] }
//    Kept for import/export so a reference PS checkpoint can seed this runtime and vice versa.
// 2. Native sharded format: magic "PSDCKPT1", u32 version, u64 manifest_len, manifest (JSON text
//    written by the runtime: shard map, versions, optimizer kind, membership epoch...), then per
//    blob {u32 dtype, u32 rank, i64[rank] shape, u64 nbytes, u32 crc32, pad to 64 B, bytes}.
//    Written to `<path>.tmp`, fsync'd, then rename()d: a crash never leaves a torn checkpoint
//    (the reference writes in place with no checksum, §5.4 of SURVEY.md).
#pragma once
#include <ATen/ATen.h>

#include <string>
#include <tuple>
#include <vector>

namespace psd {

struct RefTensor {
  std::string name;
  std::vector<int64_t> shape;
  int32_t dtype = 0;
  at::Tensor data;  // fp32, CPU
};

void save_reference_ckpt(const std::string& path, int32_t epoch, int32_t iteration, const std::vector<std::string>& names,
                         const std::vector<std::vector<int64_t>>& shapes, const std::vector<at::Tensor>& tensors);
// returns (epoch, iteration, names, shapes, dtypes, tensors)
std::tuple<int32_t, int32_t, std::vector<std::string>, std::vector<std::vector<int64_t>>, std::vector<int32_t>,
           std::vector<at::Tensor>>
load_reference_ckpt(const std::string& path);

void save_native_ckpt(const std::string& path, const std::string& manifest, const std::vector<at::Tensor>& tensors);
std::tuple<std::string, std::vector<at::Tensor>> load_native_ckpt(const std::string& path);

uint32_t crc32(const void* data, size_t n, uint32_t seed = 0);

}  // namespace psd
