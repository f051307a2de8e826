// json.h — minimal JSON value + parser for .yalm headers (objects, arrays,
// strings, numbers, true/false/null). Replaces the reference's vendored
// nlohmann/json (vendor/json.hpp) for the one use it has: parsing the
// safetensors header (codec.cpp:151-167).
#pragma once

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace yalm {

struct Json {
	enum class Type { Null, Bool, Number, String, Array, Object };
	Type type = Type::Null;
	bool b = false;
	double num = 0.0;
	std::string str;
	std::vector<Json> arr;
	std::vector<std::pair<std::string, Json>> obj; // insertion order kept

	bool is_object() const {
		return type == Type::Object;
	}
	bool contains(const std::string &k) const {
		for (auto &kv : obj)
			if (kv.first == k)
				return true;
		return false;
	}
	const Json &at(const std::string &k) const {
		for (auto &kv : obj)
			if (kv.first == k)
				return kv.second;
		throw std::out_of_range("json: missing key " + k);
	}
	const Json &operator[](size_t i) const {
		return arr.at(i);
	}
	size_t size() const {
		return type == Type::Array ? arr.size() : obj.size();
	}
	const std::string &as_string() const {
		if (type != Type::String)
			throw std::runtime_error("json: not a string");
		return str;
	}
	// metadata helper: string value or default
	std::string value(const std::string &k, const std::string &def) const {
		for (auto &kv : obj)
			if (kv.first == k && kv.second.type == Type::String)
				return kv.second.str;
		return def;
	}

	static Json parse(const std::string &text);
};

} // namespace yalm
