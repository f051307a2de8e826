// codec.h — .yalm (safetensors) reader. Same types and behaviour as the
// reference codec (/root/reference/src/codec.h:15-50): mmap the file, parse
// the JSON header, expose zero-copy tensors.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <string>
#include <unordered_map>

#include "json.h"

namespace yalm {

typedef uint16_t f16_t;

// Order matches the reference DType (codec.h:15-25) and the C ABI codes.
enum class DType {
	F32,
	F16,
	BF16,
	F8E5M2,
	F8E4M3,
	I32,
	I16,
	I8,
	U8,
};
std::string dtype_to_string(DType dtype);
size_t dtype_size(DType dtype);

struct Tensor {
	std::string name;
	DType dtype = DType::F32;
	std::array<int, 4> shape = {0, 0, 0, 0};
	void *data = nullptr;
	size_t size = 0; // bytes

	// 0 on success (codec.cpp:58-114)
	int from_json(const std::string &name, const Json &j, void *bytes_ptr, size_t bytes_size);
};

struct YALMData {
	void *data = nullptr;
	size_t size = 0;
	Json metadata;
	std::unordered_map<std::string, Tensor> tensors;

	YALMData() = default;
	YALMData(const YALMData &) = delete;
	YALMData &operator=(const YALMData &) = delete;
	~YALMData();

	// 0 on success (codec.cpp:116-175)
	int from_file(const std::string &filename);
};

} // namespace yalm
