// wa_gguf.hpp -- GGUF v2/v3 reader (zerr0o/whisper-burn src/gguf/reader.rs).
//
// Same format rules as the reference: little-endian magic "GGUF", version 2
// or 3, u64 tensor / metadata counts, metadata values skipped by type
// (reader.rs:236-283, types 0-12, arrays recursive), tensor index entries
// {string name, u32 ndims, u64 dims[ndims] (GGUF order: fastest first), u32
// ggml type (0 F32, 1 F16, 2 Q4_0 -- anything else is an error), u64
// offset}, data section at the next 32-byte boundary (reader.rs:181-183).
// The file is memory-mapped; tensor_data() returns a pointer into it.
#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace wa {

enum GgmlType : uint32_t { kGgmlF32 = 0, kGgmlF16 = 1, kGgmlQ4_0 = 2 };

struct GgufTensor {
  std::string name;
  std::vector<uint64_t> dims;  // GGUF order (reversed w.r.t. row-major)
  uint32_t type = 0;
  uint64_t offset = 0;  // relative to the data section
  uint64_t elements() const;
  uint64_t nbytes() const;  // reader.rs:39-50
};

class GgufFile {
 public:
  GgufFile() = default;
  ~GgufFile();
  GgufFile(const GgufFile&) = delete;
  GgufFile& operator=(const GgufFile&) = delete;
  // Parses header + index; on failure returns false and sets error().
  bool open(const std::string& path);
  const std::string& error() const { return err_; }
  uint32_t version() const { return version_; }
  const std::vector<GgufTensor>& tensors() const { return tensors_; }
  const GgufTensor* find(const std::string& name) const;
  // Pointer to the tensor's bytes (nbytes() long) or nullptr if out of file.
  const uint8_t* data(const GgufTensor& t) const;
  uint64_t data_section_offset() const { return data_off_; }

 private:
  bool fail(const std::string& m);
  std::string err_;
  uint32_t version_ = 0;
  std::vector<GgufTensor> tensors_;
  std::unordered_map<std::string, size_t> index_;
  const uint8_t* map_ = nullptr;
  size_t size_ = 0;
  uint64_t data_off_ = 0;
};

}  // namespace wa
