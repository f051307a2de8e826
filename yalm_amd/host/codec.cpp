#include "codec.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <iostream>

namespace yalm {

std::string dtype_to_string(DType dtype) {
	switch (dtype) {
	case DType::F32: return "F32";
	case DType::F16: return "F16";
	case DType::BF16: return "BF16";
	case DType::F8E5M2: return "F8_E5M2";
	case DType::F8E4M3: return "F8_E4M3";
	case DType::I32: return "I32";
	case DType::I16: return "I16";
	case DType::I8: return "I8";
	case DType::U8: return "U8";
	}
	return "UNKNOWN";
}

size_t dtype_size(DType dtype) {
	switch (dtype) {
	case DType::F32:
	case DType::I32: return 4;
	case DType::F16:
	case DType::BF16:
	case DType::I16: return 2;
	case DType::F8E5M2:
	case DType::F8E4M3:
	case DType::I8:
	case DType::U8: return 1;
	}
	return 0;
}

static bool parse_dtype(const std::string &s, DType &out) {
	static const std::pair<const char *, DType> table[] = {
	    {"F32", DType::F32},         {"F16", DType::F16}, {"BF16", DType::BF16}, {"F8_E5M2", DType::F8E5M2},
	    {"F8_E4M3", DType::F8E4M3}, {"I32", DType::I32}, {"I16", DType::I16},   {"I8", DType::I8},
	    {"U8", DType::U8}};
	for (auto &e : table)
		if (s == e.first) {
			out = e.second;
			return true;
		}
	return false;
}

int Tensor::from_json(const std::string &tname, const Json &val, void *bytes_ptr, size_t bytes_size) {
	name = tname;
	if (!val.contains("dtype") || !parse_dtype(val.at("dtype").str, dtype)) {
		std::cerr << "bad dtype" << std::endl;
		return -1;
	}
	const Json &shp = val.at("shape");
	if (shp.size() > 4)
		std::cerr << "shape exceeds 4 dimensions" << std::endl;
	size_t numel = 1;
	for (size_t i = 0; i < shp.size() && i < 4; i++) {
		double v = shp[i].num;
		if (v != (double)(int)v || v < 0) {
			std::cerr << "bad shape" << std::endl;
			return -1;
		}
		shape[i] = (int)v;
		numel *= shape[i];
	}
	const Json &offs = val.at("data_offsets");
	if (offs.size() != 2)
		return -1;
	const size_t start = (size_t)offs[0].num, end = (size_t)offs[1].num;
	if (end <= start || end > bytes_size) {
		std::cerr << "bad offsets" << std::endl;
		return -1;
	}
	data = (char *)bytes_ptr + start;
	size = end - start;
	if (numel * dtype_size(dtype) != size) {
		std::cerr << "bad size" << std::endl;
		return -1;
	}
	return 0;
}

YALMData::~YALMData() {
	if (data)
		munmap(data, size);
}

int YALMData::from_file(const std::string &filename) {
	fprintf(stderr, "[yalm] loading data from file: %s\n", filename.c_str());
	int fd = open(filename.c_str(), O_RDONLY);
	if (fd == -1)
		return -1;
	struct stat st;
	if (fstat(fd, &st) != 0) {
		close(fd);
		return -1;
	}
	size = st.st_size;
	data = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
	if (data == MAP_FAILED) {
		data = nullptr;
		close(fd);
		return -1;
	}
	posix_fadvise(fd, 0, size, POSIX_FADV_SEQUENTIAL);
	close(fd);
	if (size < sizeof(uint64_t))
		return -1;
	const uint64_t json_size = *(uint64_t *)data;
	if (json_size == 0 || json_size > size - sizeof(uint64_t))
		return -1;
	const char *json_ptr = (char *)data + sizeof(uint64_t);
	void *bytes_ptr = (char *)data + sizeof(uint64_t) + json_size;
	const size_t bytes_size = size - sizeof(uint64_t) - json_size;
	Json header;
	try {
		header = Json::parse(std::string(json_ptr, json_size));
	} catch (const std::exception &e) {
		std::cerr << e.what() << std::endl;
		return -1;
	}
	for (auto &kv : header.obj) {
		if (kv.first == "__metadata__") {
			metadata = kv.second;
		} else if (tensors[kv.first].from_json(kv.first, kv.second, bytes_ptr, bytes_size) != 0) {
			return -1;
		}
	}
	return 0;
}

} // namespace yalm
