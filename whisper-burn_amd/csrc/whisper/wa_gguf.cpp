// wa_gguf.cpp -- GGUF v2/v3 reader; see wa_gguf.hpp (reader.rs:105-223).
#include "wa_gguf.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>

namespace wa {

namespace {
constexpr uint32_t kMagic = 0x46554747u;  // "GGUF" little-endian (reader.rs:13)
constexpr uint64_t kAlign = 32;           // reader.rs:14

struct Cursor {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  bool take(void* dst, size_t len) {
    if (!ok || len > n - pos) return ok = false;
    if (dst) std::memcpy(dst, p + pos, len);
    pos += len;
    return true;
  }
  template <class T>
  T get() {
    T v{};
    take(&v, sizeof(T));
    return v;
  }
  bool str(std::string* out) {  // u64 length + bytes (reader.rs:229-234)
    const uint64_t len = get<uint64_t>();
    if (!ok || len > n - pos) return ok = false;
    if (out) out->assign(reinterpret_cast<const char*>(p + pos), (size_t)len);
    pos += (size_t)len;
    return true;
  }
  bool skip_value(uint32_t type, int depth = 0) {  // reader.rs:236-283
    if (depth > 8) return ok = false;
    switch (type) {
      case 0: case 1: case 7: return take(nullptr, 1);  // u8, i8, bool
      case 2: case 3: return take(nullptr, 2);          // u16, i16
      case 4: case 5: case 6: return take(nullptr, 4);  // u32, i32, f32
      case 8: return str(nullptr);                      // string
      case 9: {                                         // array
        const uint32_t et = get<uint32_t>();
        const uint64_t cnt = get<uint64_t>();
        for (uint64_t i = 0; ok && i < cnt; ++i) skip_value(et, depth + 1);
        return ok;
      }
      case 10: case 11: case 12: return take(nullptr, 8);  // u64, i64, f64
      default: return ok = false;
    }
  }
};
}  // namespace

uint64_t GgufTensor::elements() const {
  uint64_t e = 1;
  for (uint64_t d : dims) e *= d;
  return e;
}

uint64_t GgufTensor::nbytes() const {
  switch (type) {
    case kGgmlF32: return elements() * 4;
    case kGgmlF16: return elements() * 2;
    default: return elements() / 32 * 18;  // Q4_0
  }
}

GgufFile::~GgufFile() {
  if (map_) munmap(const_cast<uint8_t*>(map_), size_);
}

bool GgufFile::fail(const std::string& m) {
  err_ = m;
  return false;
}

bool GgufFile::open(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return fail("Failed to open GGUF file: " + path);
  struct stat sb;
  if (fstat(fd, &sb) != 0 || sb.st_size < 24) {
    ::close(fd);
    return fail("Failed to parse GGUF: file too small: " + path);
  }
  size_ = (size_t)sb.st_size;
  void* m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) return fail("mmap failed: " + path);
  map_ = static_cast<const uint8_t*>(m);
  Cursor c{map_, size_};
  const uint32_t magic = c.get<uint32_t>();
  if (magic != kMagic) {
    char b[96];
    snprintf(b, sizeof(b), "Invalid GGUF magic: 0x%08X (expected 0x%08X)", magic, kMagic);
    return fail(b);
  }
  version_ = c.get<uint32_t>();
  if (version_ != 2 && version_ != 3)
    return fail("Unsupported GGUF version: " + std::to_string(version_) + " (expected 2 or 3)");
  const uint64_t n_tensors = c.get<uint64_t>();
  const uint64_t n_kv = c.get<uint64_t>();
  for (uint64_t i = 0; c.ok && i < n_kv; ++i) {
    c.str(nullptr);
    const uint32_t vt = c.get<uint32_t>();
    if (c.ok && !c.skip_value(vt)) return fail("Failed to skip metadata value " + std::to_string(i));
  }
  if (!c.ok) return fail("Truncated GGUF metadata");
  if (n_tensors > size_ / 24) return fail("Corrupt GGUF tensor count");
  tensors_.reserve((size_t)n_tensors);
  for (uint64_t i = 0; i < n_tensors; ++i) {
    GgufTensor t;
    if (!c.str(&t.name)) return fail("Failed to read tensor name " + std::to_string(i));
    const uint32_t nd = c.get<uint32_t>();
    if (!c.ok || nd > 8) return fail("Failed to read ndims for tensor " + std::to_string(i));
    for (uint32_t d = 0; d < nd; ++d) t.dims.push_back(c.get<uint64_t>());
    t.type = c.get<uint32_t>();
    t.offset = c.get<uint64_t>();
    if (!c.ok) return fail("Truncated tensor index entry " + std::to_string(i));
    if (t.type > 2) return fail("Unsupported GGML dtype code: " + std::to_string(t.type));
    index_[t.name] = tensors_.size();
    tensors_.push_back(std::move(t));
  }
  data_off_ = (c.pos + kAlign - 1) / kAlign * kAlign;
  return true;
}

const GgufTensor* GgufFile::find(const std::string& name) const {
  auto it = index_.find(name);
  return it == index_.end() ? nullptr : &tensors_[it->second];
}

const uint8_t* GgufFile::data(const GgufTensor& t) const {
  const uint64_t a = data_off_ + t.offset, n = t.nbytes();
  if (a > size_ || n > size_ - a) return nullptr;
  return map_ + a;
}

}  // namespace wa
