#include "json.h"

#include <cstdlib>

namespace yalm {
namespace {

struct Parser {
	const std::string &s;
	size_t i = 0;

	[[noreturn]] void fail(const char *what) {
		throw std::runtime_error(std::string("json parse error: ") + what + " at offset " + std::to_string(i));
	}
	void ws() {
		while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t'))
			++i;
	}
	bool lit(const char *w) {
		size_t n = std::char_traits<char>::length(w);
		if (s.compare(i, n, w) == 0) {
			i += n;
			return true;
		}
		return false;
	}
	static void put_utf8(std::string &o, unsigned cp) {
		if (cp < 0x80) {
			o += (char)cp;
		} else if (cp < 0x800) {
			o += (char)(0xC0 | (cp >> 6));
			o += (char)(0x80 | (cp & 0x3F));
		} else if (cp < 0x10000) {
			o += (char)(0xE0 | (cp >> 12));
			o += (char)(0x80 | ((cp >> 6) & 0x3F));
			o += (char)(0x80 | (cp & 0x3F));
		} else {
			o += (char)(0xF0 | (cp >> 18));
			o += (char)(0x80 | ((cp >> 12) & 0x3F));
			o += (char)(0x80 | ((cp >> 6) & 0x3F));
			o += (char)(0x80 | (cp & 0x3F));
		}
	}
	unsigned hex4() {
		if (i + 4 > s.size())
			fail("short \\u escape");
		unsigned v = (unsigned)std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
		i += 4;
		return v;
	}
	std::string string() {
		if (s[i] != '"')
			fail("expected string");
		++i;
		std::string o;
		while (i < s.size() && s[i] != '"') {
			char c = s[i++];
			if (c != '\\') {
				o += c;
				continue;
			}
			if (i >= s.size())
				fail("bad escape");
			char e = s[i++];
			switch (e) {
			case '"': o += '"'; break;
			case '\\': o += '\\'; break;
			case '/': o += '/'; break;
			case 'b': o += '\b'; break;
			case 'f': o += '\f'; break;
			case 'n': o += '\n'; break;
			case 'r': o += '\r'; break;
			case 't': o += '\t'; break;
			case 'u': {
				unsigned cp = hex4();
				if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
					i += 2;
					unsigned lo = hex4();
					cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
				}
				put_utf8(o, cp);
				break;
			}
			default:
				fail("bad escape");
			}
		}
		if (i >= s.size())
			fail("unterminated string");
		++i;
		return o;
	}
	Json value() {
		ws();
		if (i >= s.size())
			fail("unexpected end");
		Json j;
		char c = s[i];
		if (c == '{') {
			j.type = Json::Type::Object;
			++i;
			ws();
			if (s[i] == '}') {
				++i;
				return j;
			}
			while (true) {
				ws();
				std::string k = string();
				ws();
				if (s[i] != ':')
					fail("expected ':'");
				++i;
				j.obj.emplace_back(std::move(k), value());
				ws();
				if (s[i] == ',') {
					++i;
					continue;
				}
				if (s[i] == '}') {
					++i;
					return j;
				}
				fail("expected ',' or '}'");
			}
		}
		if (c == '[') {
			j.type = Json::Type::Array;
			++i;
			ws();
			if (s[i] == ']') {
				++i;
				return j;
			}
			while (true) {
				j.arr.push_back(value());
				ws();
				if (s[i] == ',') {
					++i;
					continue;
				}
				if (s[i] == ']') {
					++i;
					return j;
				}
				fail("expected ',' or ']'");
			}
		}
		if (c == '"') {
			j.type = Json::Type::String;
			j.str = string();
			return j;
		}
		if (lit("true")) {
			j.type = Json::Type::Bool;
			j.b = true;
			return j;
		}
		if (lit("false")) {
			j.type = Json::Type::Bool;
			return j;
		}
		if (lit("null"))
			return j;
		char *end = nullptr;
		j.num = std::strtod(s.c_str() + i, &end);
		if (end == s.c_str() + i)
			fail("bad value");
		i = end - s.c_str();
		j.type = Json::Type::Number;
		return j;
	}
};

} // namespace

Json Json::parse(const std::string &text) {
	Parser p{text};
	Json j = p.value();
	p.ws();
	if (p.i != text.size())
		p.fail("trailing characters");
	return j;
}

} // namespace yalm
