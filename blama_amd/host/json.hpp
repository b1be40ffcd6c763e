// A small JSON value with a parser and a serializer, enough for Blama's wire format
// (server/code/http/HttpServerMain.cpp: /complete and /verify_completion bodies).  The
// reference uses nlohmann::json, which is not in this image.  Numbers are doubles.  A float
// logit is written with 9 significant digits, which parses back to the same float: the
// verify round trip depends on that.  Strings that are not valid UTF-8 (a byte-fallback token
// such as <0xE2> on its own) are written with U+FFFD for each maximal invalid subpart, the
// Unicode-recommended practice (and Python's errors="replace").  nlohmann's default dump
// throws on them instead, which ends the reference's request.
#pragma once
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace bl::json {

struct Value {
    enum class Kind { Null, Bool, Number, String, Array, Object };
    Kind kind = Kind::Null;
    bool b = false;
    double num = 0.0;
    bool num_is_float = false;          // print with float precision (logits)
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;   // insertion order kept

    Value() = default;
    static Value number(double v, bool as_float = false) {
        Value x;
        x.kind = Kind::Number;
        x.num = v;
        x.num_is_float = as_float;
        return x;
    }
    static Value string(std::string s) {
        Value x;
        x.kind = Kind::String;
        x.str = std::move(s);
        return x;
    }
    static Value array() {
        Value x;
        x.kind = Kind::Array;
        return x;
    }
    static Value object() {
        Value x;
        x.kind = Kind::Object;
        return x;
    }
    bool is_object() const { return kind == Kind::Object; }
    bool is_array() const { return kind == Kind::Array; }
    const Value* find(std::string_view k) const {
        for (auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    const Value& at(std::string_view k) const {
        const Value* v = find(k);
        if (!v) throw std::runtime_error("json: missing key \"" + std::string(k) + "\"");
        return *v;
    }
    Value& set(const std::string& k, Value v) {
        for (auto& kv : obj)
            if (kv.first == k) return kv.second = std::move(v);
        obj.emplace_back(k, std::move(v));
        return obj.back().second;
    }
    double as_number() const {
        if (kind != Kind::Number) throw std::runtime_error("json: not a number");
        return num;
    }
    const std::string& as_string() const {
        if (kind != Kind::String) throw std::runtime_error("json: not a string");
        return str;
    }
};

namespace detail {
struct Parser {
    std::string_view s;
    size_t i = 0;
    int depth = 0;
    static constexpr int kMaxDepth = 256;   // nesting bound: no stack overflow on "[[[[..."
    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("json parse error: ") + what + " at " + std::to_string(i));
    }
    void ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool lit(std::string_view w) {
        if (s.substr(i, w.size()) == w) {
            i += w.size();
            return true;
        }
        return false;
    }
    static void utf8(std::string& o, unsigned cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        }
    }
    unsigned hex4() {
        if (i + 4 > s.size()) fail("short \\u escape");
        unsigned v = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = s[i++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else fail("bad \\u escape");
        }
        return v;
    }
    std::string str() {
        if (s[i] != '"') fail("expected string");
        ++i;
        std::string o;
        while (i < s.size() && s[i] != '"') {
            char c = s[i++];
            if (c != '\\') { o += c; continue; }
            if (i >= s.size()) fail("bad escape");
            c = s[i++];
            switch (c) {
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
                if (cp >= 0xD800 && cp < 0xDC00 && lit("\\u")) cp = 0x10000 + ((cp - 0xD800) << 10) + (hex4() - 0xDC00);
                utf8(o, cp);
                break;
            }
            default: fail("bad escape");
            }
        }
        if (i >= s.size()) fail("unterminated string");
        ++i;
        return o;
    }
    // A JSON number (RFC 8259 grammar: no nan/inf/hex/leading '+'), finite after conversion.
    Value number() {
        const size_t b = i;
        if (i < s.size() && s[i] == '-') ++i;
        auto digits = [&] { size_t k = i; while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i; return i - k; };
        if (i < s.size() && s[i] == '0') ++i;
        else if (digits() == 0) fail("bad value");
        if (i < s.size() && s[i] == '.') { ++i; if (digits() == 0) fail("bad number"); }
        if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
            ++i;
            if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
            if (digits() == 0) fail("bad number");
        }
        const std::string tok(s.substr(b, i - b));
        const double d = std::strtod(tok.c_str(), nullptr);
        if (!std::isfinite(d)) fail("number out of range");
        return Value::number(d);
    }
    struct DepthGuard {
        Parser& p;
        explicit DepthGuard(Parser& q) : p(q) { if (++p.depth > kMaxDepth) p.fail("nesting too deep"); }
        ~DepthGuard() { --p.depth; }
    };
    Value val() {
        ws();
        if (i >= s.size()) fail("unexpected end");
        const char c = s[i];
        DepthGuard guard(*this);
        if (c == '{') {
            ++i;
            Value o = Value::object();
            ws();
            if (i < s.size() && s[i] == '}') { ++i; return o; }
            while (true) {
                ws();
                std::string k = str();
                ws();
                if (i >= s.size() || s[i] != ':') fail("expected ':'");
                ++i;
                o.set(k, val());
                ws();
                if (i < s.size() && s[i] == ',') { ++i; continue; }
                if (i < s.size() && s[i] == '}') { ++i; return o; }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            ++i;
            Value a = Value::array();
            ws();
            if (i < s.size() && s[i] == ']') { ++i; return a; }
            while (true) {
                a.arr.push_back(val());
                ws();
                if (i < s.size() && s[i] == ',') { ++i; continue; }
                if (i < s.size() && s[i] == ']') { ++i; return a; }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') return Value::string(str());
        if (lit("true")) { Value v; v.kind = Value::Kind::Bool; v.b = true; return v; }
        if (lit("false")) { Value v; v.kind = Value::Kind::Bool; return v; }
        if (lit("null")) return Value();
        return number();
    }
};

// Length of the valid UTF-8 sequence at s[i], or -(bytes of its maximal invalid subpart).
inline int utf8_seq(const std::string& s, size_t i) {
    const unsigned char b = (unsigned char)s[i];
    if (b < 0x80) return 1;
    int n;
    unsigned char lo = 0x80, hi = 0xBF;
    if (b >= 0xC2 && b <= 0xDF) n = 2;
    else if (b >= 0xE0 && b <= 0xEF) { n = 3; if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; }
    else if (b >= 0xF0 && b <= 0xF4) { n = 4; if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; }
    else return -1;
    for (int k = 1; k < n; ++k) {
        if (i + k >= s.size()) return -k;
        const unsigned char c = (unsigned char)s[i + k];
        if (c < (k == 1 ? lo : 0x80) || c > (k == 1 ? hi : 0xBF)) return -k;
    }
    return n;
}

inline void dump_str(std::string& o, const std::string& s) {
    o += '"';
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = (unsigned char)s[i];
        if (c >= 0x80) {
            const int n = utf8_seq(s, i);
            if (n > 0) o.append(s, i, (size_t)n);
            else o += "\xEF\xBF\xBD";
            i += (size_t)(n > 0 ? n : -n);
            continue;
        }
        ++i;
        switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        default:
            if (c < 0x20) {
                char buf[8];
                std::snprintf(buf, sizeof buf, "\\u%04x", c);
                o += buf;
            } else {
                o += (char)c;
            }
        }
    }
    o += '"';
}

inline void dump(std::string& o, const Value& v) {
    switch (v.kind) {
    case Value::Kind::Null: o += "null"; break;
    case Value::Kind::Bool: o += v.b ? "true" : "false"; break;
    case Value::Kind::Number: {
        char buf[40];
        if (v.num == std::floor(v.num) && std::fabs(v.num) < 1e15 && !v.num_is_float)
            std::snprintf(buf, sizeof buf, "%lld", (long long)v.num);
        else
            std::snprintf(buf, sizeof buf, v.num_is_float ? "%.9g" : "%.17g", v.num);
        o += buf;
        break;
    }
    case Value::Kind::String: dump_str(o, v.str); break;
    case Value::Kind::Array:
        o += '[';
        for (size_t k = 0; k < v.arr.size(); ++k) {
            if (k) o += ',';
            dump(o, v.arr[k]);
        }
        o += ']';
        break;
    case Value::Kind::Object:
        o += '{';
        for (size_t k = 0; k < v.obj.size(); ++k) {
            if (k) o += ',';
            dump_str(o, v.obj[k].first);
            o += ':';
            dump(o, v.obj[k].second);
        }
        o += '}';
        break;
    }
}
}  // namespace detail

inline Value parse(std::string_view text) {
    detail::Parser p{text};
    Value v = p.val();
    p.ws();
    if (p.i != text.size()) p.fail("trailing characters");
    return v;
}

inline std::string dump(const Value& v) {
    std::string o;
    detail::dump(o, v);
    return o;
}

}  // namespace bl::json
