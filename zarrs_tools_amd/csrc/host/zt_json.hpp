// zt_json.hpp — a small JSON value, parser and writer for Zarr V3 metadata (zarr.json) and the
// zarrs_filter run configs. Objects keep insertion order so written metadata reads naturally.
#pragma once

#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace zt {
namespace json {

struct Value;
using Object = std::vector<std::pair<std::string, Value>>;
using Array = std::vector<Value>;

struct Value {
    enum Kind { Null, Bool, Int, Double, String, Arr, Obj } kind = Null;
    bool b = false;
    int64_t i = 0;
    double d = 0.0;
    std::string s;
    std::shared_ptr<Array> a;
    std::shared_ptr<Object> o;

    Value() = default;
    Value(std::nullptr_t) {}
    Value(bool v) : kind(Bool), b(v) {}
    Value(int v) : kind(Int), i(v) {}
    Value(int64_t v) : kind(Int), i(v) {}
    Value(uint64_t v) : kind(Int), i((int64_t)v) {}
    Value(double v) : kind(Double), d(v) {}
    Value(const char* v) : kind(String), s(v) {}
    Value(std::string v) : kind(String), s(std::move(v)) {}
    Value(Array v) : kind(Arr), a(std::make_shared<Array>(std::move(v))) {}
    Value(Object v) : kind(Obj), o(std::make_shared<Object>(std::move(v))) {}

    bool is_null() const { return kind == Null; }
    bool is_num() const { return kind == Int || kind == Double; }
    bool is_str() const { return kind == String; }
    bool is_obj() const { return kind == Obj; }
    bool is_arr() const { return kind == Arr; }

    const Value* find(const std::string& k) const {
        if (kind != Obj) return nullptr;
        for (auto& kv : *o)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    const Value& at(const std::string& k) const {
        const Value* v = find(k);
        if (!v) throw std::runtime_error("missing key \"" + k + "\"");
        return *v;
    }
    void set(const std::string& k, Value v) {
        if (kind != Obj) { kind = Obj; o = std::make_shared<Object>(); }
        for (auto& kv : *o)
            if (kv.first == k) { kv.second = std::move(v); return; }
        o->emplace_back(k, std::move(v));
    }
    const Array& arr() const {
        if (kind != Arr) throw std::runtime_error("expected a JSON array");
        return *a;
    }
    const std::string& str() const {
        if (kind != String) throw std::runtime_error("expected a JSON string");
        return s;
    }
    int64_t as_int() const {
        if (kind == Int) return i;
        if (kind == Double && std::floor(d) == d) return (int64_t)d;
        throw std::runtime_error("expected an integer");
    }
    double as_double() const {
        if (kind == Int) return (double)i;
        if (kind == Double) return d;
        throw std::runtime_error("expected a number");
    }
};

class Parser {
  public:
    explicit Parser(const std::string& t) : t_(t) {}
    Value parse() {
        Value v = value();
        ws();
        if (p_ != t_.size()) err("trailing characters");
        return v;
    }

  private:
    const std::string& t_;
    size_t p_ = 0;

    [[noreturn]] void err(const char* what) {
        throw std::runtime_error(std::string("JSON: ") + what + " at offset " + std::to_string(p_));
    }
    void ws() {
        while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\r' || t_[p_] == '\t'))
            ++p_;
    }
    bool lit(const char* w) {
        size_t n = std::char_traits<char>::length(w);
        if (t_.compare(p_, n, w) == 0) { p_ += n; return true; }
        return false;
    }
    Value value() {
        ws();
        if (p_ >= t_.size()) err("unexpected end");
        char c = t_[p_];
        if (c == '{') return object();
        if (c == '[') return array();
        if (c == '"') return Value(string());
        if (lit("true")) return Value(true);
        if (lit("false")) return Value(false);
        if (lit("null")) return Value();
        return number();
    }
    Value object() {
        ++p_;
        Object o;
        ws();
        if (p_ < t_.size() && t_[p_] == '}') { ++p_; return Value(std::move(o)); }
        for (;;) {
            ws();
            if (p_ >= t_.size() || t_[p_] != '"') err("expected a key");
            std::string k = string();
            ws();
            if (p_ >= t_.size() || t_[p_] != ':') err("expected ':'");
            ++p_;
            o.emplace_back(std::move(k), value());
            ws();
            if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
            if (p_ < t_.size() && t_[p_] == '}') { ++p_; break; }
            err("expected ',' or '}'");
        }
        return Value(std::move(o));
    }
    Value array() {
        ++p_;
        Array a;
        ws();
        if (p_ < t_.size() && t_[p_] == ']') { ++p_; return Value(std::move(a)); }
        for (;;) {
            a.push_back(value());
            ws();
            if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
            if (p_ < t_.size() && t_[p_] == ']') { ++p_; break; }
            err("expected ',' or ']'");
        }
        return Value(std::move(a));
    }
    static void utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) out += (char)cp;
        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F));
            out += (char)(0x80 | (cp & 0x3F));
        } else {
            out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
            out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
        }
    }
    uint32_t hex4() {
        if (p_ + 4 > t_.size()) err("bad \\u escape");
        uint32_t v = (uint32_t)std::strtoul(t_.substr(p_, 4).c_str(), nullptr, 16);
        p_ += 4;
        return v;
    }
    std::string string() {
        ++p_;
        std::string out;
        while (p_ < t_.size() && t_[p_] != '"') {
            char c = t_[p_++];
            if (c != '\\') { out += c; continue; }
            if (p_ >= t_.size()) err("bad escape");
            char e = t_[p_++];
            switch (e) {
            case '"': out += '"'; break;
            case '\\': out += '\\'; break;
            case '/': out += '/'; break;
            case 'b': out += '\b'; break;
            case 'f': out += '\f'; break;
            case 'n': out += '\n'; break;
            case 'r': out += '\r'; break;
            case 't': out += '\t'; break;
            case 'u': {
                uint32_t cp = hex4();
                if (cp >= 0xD800 && cp < 0xDC00 && t_.compare(p_, 2, "\\u") == 0) {
                    p_ += 2;
                    uint32_t lo = hex4();
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                }
                utf8(out, cp);
                break;
            }
            default: err("bad escape");
            }
        }
        if (p_ >= t_.size()) err("unterminated string");
        ++p_;
        return out;
    }
    Value number() {
        size_t b = p_;
        bool flt = false;
        if (p_ < t_.size() && (t_[p_] == '-' || t_[p_] == '+')) ++p_;
        while (p_ < t_.size()) {
            char c = t_[p_];
            if (c >= '0' && c <= '9') { ++p_; continue; }
            if (c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-') { flt = true; ++p_; continue; }
            break;
        }
        if (b == p_) err("unexpected character");
        std::string num = t_.substr(b, p_ - b);
        if (!flt) {
            errno = 0;
            long long v = std::strtoll(num.c_str(), nullptr, 10);
            if (errno == 0) return Value((int64_t)v);
            return Value((uint64_t)std::strtoull(num.c_str(), nullptr, 10));
        }
        return Value(std::strtod(num.c_str(), nullptr));
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

inline void escape(std::string& out, const std::string& s) {
    out += '"';
    for (unsigned char c : s) {
        switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        default:
            if (c < 0x20) {
                char buf[8];
                std::snprintf(buf, sizeof(buf), "\\u%04x", c);
                out += buf;
            } else {
                out += (char)c;
            }
        }
    }
    out += '"';
}

inline void dump(std::string& out, const Value& v, int indent, int level) {
    auto nl = [&](int lv) {
        if (indent < 0) return;
        out += '\n';
        out.append((size_t)(indent * lv), ' ');
    };
    switch (v.kind) {
    case Value::Null: out += "null"; break;
    case Value::Bool: out += v.b ? "true" : "false"; break;
    case Value::Int: out += std::to_string(v.i); break;
    case Value::Double: {
        if (std::isnan(v.d)) { out += "\"NaN\""; break; }
        if (std::isinf(v.d)) { out += v.d > 0 ? "\"Infinity\"" : "\"-Infinity\""; break; }
        char buf[40];
        std::snprintf(buf, sizeof(buf), "%.17g", v.d);
        std::string t(buf);
        if (t.find_first_of(".eE") == std::string::npos) t += ".0";
        out += t;
        break;
    }
    case Value::String: escape(out, v.s); break;
    case Value::Arr: {
        // short numeric arrays on one line (shapes), everything else one element per line
        bool flat = true;
        for (auto& e : *v.a) flat = flat && (e.kind == Value::Int || e.kind == Value::Double);
        out += '[';
        for (size_t k = 0; k < v.a->size(); ++k) {
            if (k) out += flat ? ", " : ",";
            if (!flat) nl(level + 1);
            dump(out, (*v.a)[k], indent, level + 1);
        }
        if (!flat && !v.a->empty()) nl(level);
        out += ']';
        break;
    }
    case Value::Obj: {
        out += '{';
        for (size_t k = 0; k < v.o->size(); ++k) {
            if (k) out += ',';
            nl(level + 1);
            escape(out, (*v.o)[k].first);
            out += indent < 0 ? ":" : ": ";
            dump(out, (*v.o)[k].second, indent, level + 1);
        }
        if (!v.o->empty()) nl(level);
        out += '}';
        break;
    }
    }
}

inline std::string dump(const Value& v, int indent = 2) {
    std::string out;
    dump(out, v, indent, 0);
    return out;
}

}  // namespace json
}  // namespace zt
