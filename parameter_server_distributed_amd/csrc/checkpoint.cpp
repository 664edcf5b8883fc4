#include "checkpoint.h"

#include <fcntl.h>
#include <unistd.h>

#include <array>
#include <cstdio>
#include <cstring>
#include <fstream>

namespace psd {

namespace {

std::array<uint32_t, 256> make_crc_table() {
  std::array<uint32_t, 256> t{};
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
    t[i] = c;
  }
  return t;
}

struct FileWriter {
  FILE* f = nullptr;
  std::string path, tmp;
  explicit FileWriter(const std::string& p) : path(p), tmp(p + ".tmp") {
    f = std::fopen(tmp.c_str(), "wb");
    TORCH_CHECK(f, "psd: cannot open ", tmp, " for writing");
  }
  void write(const void* d, size_t n) { TORCH_CHECK(std::fwrite(d, 1, n, f) == n, "psd: short write to ", tmp); }
  template <typename T>
  void pod(const T& v) { write(&v, sizeof(T)); }
  void commit() {
    TORCH_CHECK(std::fflush(f) == 0, "psd: fflush failed for ", tmp);
    TORCH_CHECK(::fsync(fileno(f)) == 0, "psd: fsync failed for ", tmp);
    std::fclose(f);
    f = nullptr;
    TORCH_CHECK(std::rename(tmp.c_str(), path.c_str()) == 0, "psd: rename ", tmp, " -> ", path, " failed");
  }
  ~FileWriter() {
    if (f) {
      std::fclose(f);
      std::remove(tmp.c_str());
    }
  }
};

struct FileReader {
  std::ifstream in;
  std::string path;
  explicit FileReader(const std::string& p) : in(p, std::ios::binary), path(p) {
    TORCH_CHECK(in.is_open(), "psd: cannot open checkpoint ", p);
  }
  void read(void* d, size_t n) {
    in.read(static_cast<char*>(d), (std::streamsize)n);
    TORCH_CHECK((size_t)in.gcount() == n, "psd: truncated checkpoint ", path);
  }
  template <typename T>
  T pod() {
    T v;
    read(&v, sizeof(T));
    return v;
  }
};

at::Tensor cpu_contig(const at::Tensor& t) { return t.detach().to(at::kCPU).contiguous(); }

}  // namespace

uint32_t crc32(const void* data, size_t n, uint32_t seed) {
  static const std::array<uint32_t, 256> table = make_crc_table();
  uint32_t c = seed ^ 0xFFFFFFFFu;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

void save_reference_ckpt(const std::string& path, int32_t epoch, int32_t iteration, const std::vector<std::string>& names,
                         const std::vector<std::vector<int64_t>>& shapes, const std::vector<at::Tensor>& tensors) {
  TORCH_CHECK(names.size() == tensors.size() && shapes.size() == tensors.size(), "psd: ckpt list length mismatch");
  FileWriter w(path);
  w.pod<int32_t>(epoch);
  w.pod<int32_t>(iteration);
  w.pod<uint64_t>(tensors.size());
  for (size_t i = 0; i < tensors.size(); ++i) {
    w.pod<uint64_t>(names[i].size());
    w.write(names[i].data(), names[i].size());
    w.pod<uint64_t>(shapes[i].size());
    for (int64_t d : shapes[i]) w.pod<int32_t>((int32_t)d);
    w.pod<int32_t>(0);  // dtype: always fp32 payload, as in the reference
    at::Tensor t = cpu_contig(tensors[i]).to(at::kFloat);
    w.pod<uint64_t>((uint64_t)t.numel());
    w.write(t.data_ptr<float>(), (size_t)t.numel() * sizeof(float));
  }
  w.commit();
}

std::tuple<int32_t, int32_t, std::vector<std::string>, std::vector<std::vector<int64_t>>, std::vector<int32_t>,
           std::vector<at::Tensor>>
load_reference_ckpt(const std::string& path) {
  FileReader r(path);
  int32_t epoch = r.pod<int32_t>();
  int32_t iteration = r.pod<int32_t>();
  uint64_t n = r.pod<uint64_t>();
  TORCH_CHECK(n < (1ull << 24), "psd: implausible tensor count in ", path);
  std::vector<std::string> names;
  std::vector<std::vector<int64_t>> shapes;
  std::vector<int32_t> dtypes;
  std::vector<at::Tensor> data;
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t nl = r.pod<uint64_t>();
    TORCH_CHECK(nl < (1ull << 20), "psd: implausible name length in ", path);
    std::string name(nl, '\0');
    r.read(name.data(), nl);
    uint64_t rank = r.pod<uint64_t>();
    TORCH_CHECK(rank < 64, "psd: implausible rank in ", path);
    std::vector<int64_t> shape(rank);
    for (uint64_t d = 0; d < rank; ++d) shape[d] = r.pod<int32_t>();
    int32_t dt = r.pod<int32_t>();
    uint64_t numel = r.pod<uint64_t>();
    at::Tensor t = at::empty({(int64_t)numel}, at::kFloat);
    r.read(t.data_ptr<float>(), numel * sizeof(float));
    names.push_back(std::move(name));
    shapes.push_back(std::move(shape));
    dtypes.push_back(dt);
    data.push_back(t);
  }
  return {epoch, iteration, names, shapes, dtypes, data};
}

static constexpr char kMagic[8] = {'P', 'S', 'D', 'C', 'K', 'P', 'T', '1'};

static int32_t code_of(at::ScalarType s) {
  switch (s) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kFloat8_e4m3fn: return 2;
    case at::kInt: return 3;
    case at::kLong: return 4;
    case at::kByte: return 5;
    case at::kDouble: return 6;
    default: TORCH_CHECK(false, "psd: dtype not checkpointable: ", s);
  }
}
static at::ScalarType type_of(int32_t c) {
  static const at::ScalarType m[] = {at::kFloat, at::kBFloat16, at::kFloat8_e4m3fn, at::kInt,
                                     at::kLong,  at::kByte,     at::kDouble};
  TORCH_CHECK(c >= 0 && c < 7, "psd: bad dtype code in checkpoint");
  return m[c];
}

void save_native_ckpt(const std::string& path, const std::string& manifest, const std::vector<at::Tensor>& tensors) {
  FileWriter w(path);
  w.write(kMagic, 8);
  w.pod<uint32_t>(1);
  w.pod<uint64_t>(manifest.size());
  w.write(manifest.data(), manifest.size());
  w.pod<uint64_t>(tensors.size());
  uint64_t pos = 8 + 4 + 8 + manifest.size() + 8;
  static const char zeros[64] = {0};
  for (const auto& t0 : tensors) {
    at::Tensor t = cpu_contig(t0);
    const uint64_t nbytes = (uint64_t)t.numel() * t.element_size();
    w.pod<uint32_t>((uint32_t)code_of(t.scalar_type()));
    w.pod<uint32_t>((uint32_t)t.dim());
    for (int64_t d : t.sizes()) w.pod<int64_t>(d);
    w.pod<uint64_t>(nbytes);
    w.pod<uint32_t>(crc32(t.data_ptr(), nbytes));
    pos += 4 + 4 + 8 * t.dim() + 8 + 4;
    const uint64_t pad = (64 - pos % 64) % 64;
    w.write(zeros, pad);
    pos += pad;
    w.write(t.data_ptr(), nbytes);
    pos += nbytes;
  }
  w.commit();
}

std::tuple<std::string, std::vector<at::Tensor>> load_native_ckpt(const std::string& path) {
  FileReader r(path);
  char magic[8];
  r.read(magic, 8);
  TORCH_CHECK(std::memcmp(magic, kMagic, 8) == 0, "psd: ", path, " is not a native checkpoint");
  uint32_t ver = r.pod<uint32_t>();
  TORCH_CHECK(ver == 1, "psd: unsupported checkpoint version ", ver);
  uint64_t ml = r.pod<uint64_t>();
  std::string manifest(ml, '\0');
  r.read(manifest.data(), ml);
  uint64_t n = r.pod<uint64_t>();
  uint64_t pos = 8 + 4 + 8 + ml + 8;
  std::vector<at::Tensor> out;
  for (uint64_t i = 0; i < n; ++i) {
    int32_t code = (int32_t)r.pod<uint32_t>();
    uint32_t rank = r.pod<uint32_t>();
    TORCH_CHECK(rank < 64, "psd: corrupt checkpoint (rank)");
    std::vector<int64_t> shape(rank);
    for (uint32_t d = 0; d < rank; ++d) shape[d] = r.pod<int64_t>();
    uint64_t nbytes = r.pod<uint64_t>();
    uint32_t crc = r.pod<uint32_t>();
    pos += 4 + 4 + 8 * rank + 8 + 4;
    const uint64_t pad = (64 - pos % 64) % 64;
    char skip[64];
    r.read(skip, pad);
    pos += pad;
    at::Tensor t = at::empty(shape, at::TensorOptions().dtype(type_of(code)));
    TORCH_CHECK((uint64_t)t.numel() * t.element_size() == nbytes, "psd: corrupt checkpoint (size)");
    r.read(t.data_ptr(), nbytes);
    pos += nbytes;
    TORCH_CHECK(crc32(t.data_ptr(), nbytes) == crc, "psd: checksum mismatch in ", path, " blob ", i);
    out.push_back(t);
  }
  return {manifest, out};
}

}  // namespace psd
