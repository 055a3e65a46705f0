// TEST INFRASTRUCTURE — part of the CPU oracle (oracle/), never linked into the product.
//
// A small model of JavaScript values as they flow through the reference merge-tree:
// JSON.parse / JSON.stringify (V8 7.8 semantics, as used by Node 12 and by the reference's
// TestSerializer, merge-tree/src/test/testSerializer.ts:27-30), JS object key order
// (integer-like keys first, ascending, then insertion order), UTF-16 strings.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace orc {

using u16s = std::u16string;

struct JV;
using JVP = std::shared_ptr<JV>;

// JS array-index test: canonical decimal in [0, 2^32-2]; such keys enumerate first, ascending.
inline bool is_array_index(const u16s& k, uint32_t* out = nullptr) {
    if (k.empty() || k.size() > 10) return false;
    if (k[0] == u'0' && k.size() > 1) return false;
    uint64_t v = 0;
    for (char16_t c : k) {
        if (c < u'0' || c > u'9') return false;
        v = v * 10 + (c - u'0');
    }
    if (v > 4294967294ull) return false;
    if (out) *out = (uint32_t)v;
    return true;
}

// Insertion-ordered JS object. keys() returns JS enumeration order.
struct JObj {
    std::vector<std::pair<u16s, JVP>> ents;
    JVP get(const u16s& k) const {
        for (auto& e : ents)
            if (e.first == k) return e.second;
        return nullptr;
    }
    void set(const u16s& k, JVP v) {
        for (auto& e : ents)
            if (e.first == k) { e.second = std::move(v); return; }
        ents.emplace_back(k, std::move(v));
    }
    bool del(const u16s& k) {
        for (size_t i = 0; i < ents.size(); i++)
            if (ents[i].first == k) { ents.erase(ents.begin() + i); return true; }
        return false;
    }
    std::vector<u16s> keys() const {
        std::vector<std::pair<uint32_t, u16s>> ints;
        std::vector<u16s> strs;
        for (auto& e : ents) {
            uint32_t idx;
            if (is_array_index(e.first, &idx)) ints.emplace_back(idx, e.first);
            else strs.push_back(e.first);
        }
        std::sort(ints.begin(), ints.end(), [](auto& a, auto& b) { return a.first < b.first; });
        std::vector<u16s> out;
        for (auto& p : ints) out.push_back(p.second);
        for (auto& s : strs) out.push_back(s);
        return out;
    }
};

struct JV {
    enum T { Null, Bool, Num, Str, Arr, Obj } t = Null;
    bool b = false;
    double n = 0;
    u16s s;
    std::vector<JVP> a;
    JObj o;
    static JVP null() { return std::make_shared<JV>(); }
    static JVP num(double v) { auto p = std::make_shared<JV>(); p->t = Num; p->n = v; return p; }
    static JVP str(const u16s& v) { auto p = std::make_shared<JV>(); p->t = Str; p->s = v; return p; }
    static JVP boolean(bool v) { auto p = std::make_shared<JV>(); p->t = Bool; p->b = v; return p; }
    static JVP obj() { auto p = std::make_shared<JV>(); p->t = Obj; return p; }
};

// ---- UTF-8 <-> UTF-16 ----------------------------------------------------------------------
inline u16s utf8_to_u16(const char* s, size_t n) {
    u16s out;
    size_t i = 0;
    while (i < n) {
        uint32_t c = (uint8_t)s[i];
        uint32_t cp;
        int len;
        if (c < 0x80) { cp = c; len = 1; }
        else if ((c >> 5) == 6) { cp = c & 0x1f; len = 2; }
        else if ((c >> 4) == 14) { cp = c & 0x0f; len = 3; }
        else { cp = c & 0x07; len = 4; }
        for (int k = 1; k < len && i + k < n; k++) cp = (cp << 6) | ((uint8_t)s[i + k] & 0x3f);
        i += len;
        if (cp >= 0x10000) {
            cp -= 0x10000;
            out.push_back((char16_t)(0xD800 + (cp >> 10)));
            out.push_back((char16_t)(0xDC00 + (cp & 0x3ff)));
        } else {
            out.push_back((char16_t)cp);
        }
    }
    return out;
}

inline void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o.push_back((char)cp);
    else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3f))); }
    else if (cp < 0x10000) {
        o.push_back((char)(0xE0 | (cp >> 12)));
        o.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
        o.push_back((char)(0x80 | (cp & 0x3f)));
    } else {
        o.push_back((char)(0xF0 | (cp >> 18)));
        o.push_back((char)(0x80 | ((cp >> 12) & 0x3f)));
        o.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
        o.push_back((char)(0x80 | (cp & 0x3f)));
    }
}

// UTF-16 -> UTF-8; lone surrogates become U+FFFD (Node Buffer.from(str, "utf8") behaviour).
inline std::string u16_to_utf8(const u16s& s) {
    std::string o;
    o.reserve(s.size());
    for (size_t i = 0; i < s.size(); i++) {
        uint32_t c = s[i];
        if (c >= 0xD800 && c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            uint32_t cp = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
            put_utf8(o, cp);
            i++;
        } else if (c >= 0xD800 && c <= 0xDFFF) {
            put_utf8(o, 0xFFFD);
        } else {
            put_utf8(o, c);
        }
    }
    return o;
}

// ---- JSON.stringify --------------------------------------------------------------------------
// Number.prototype.toString(10) for finite doubles (ECMA-262 Number::toString, shortest digits).
inline std::string js_number(double x) {
    if (std::isnan(x) || std::isinf(x)) return "null";  // JSON.stringify
    if (x == 0) return "0";
    std::string sign;
    if (x < 0) { sign = "-"; x = -x; }
    char buf[64];
    int p;
    for (p = 1; p <= 17; p++) {
        snprintf(buf, sizeof buf, "%.*e", p - 1, x);
        if (strtod(buf, nullptr) == x) break;
    }
    // buf = d[.ddd]e[+-]XX
    std::string digits;
    const char* q = buf;
    while (*q && *q != 'e') { if (*q != '.') digits.push_back(*q); q++; }
    int e = atoi(q + 1);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    int k = (int)digits.size();
    int n = e + 1;
    std::string out;
    if (k <= n && n <= 21) {
        out = digits + std::string(n - k, '0');
    } else if (0 < n && n <= 21) {
        out = digits.substr(0, n) + "." + digits.substr(n);
    } else if (-6 < n && n <= 0) {
        out = "0." + std::string(-n, '0') + digits;
    } else {
        out = digits.substr(0, 1);
        if (k > 1) out += "." + digits.substr(1);
        out += "e";
        out += (n - 1 >= 0) ? "+" : "-";
        out += std::to_string(std::abs(n - 1));
    }
    return sign + out;
}

// JSON.stringify string quoting (well-formed JSON.stringify, V8 >= 7.2).
inline void js_quote(std::string& o, const u16s& s) {
    static const char* hex = "0123456789abcdef";
    o.push_back('"');
    for (size_t i = 0; i < s.size(); i++) {
        uint32_t c = s[i];
        switch (c) {
            case '"': o += "\\\""; continue;
            case '\\': o += "\\\\"; continue;
            case '\b': o += "\\b"; continue;
            case '\f': o += "\\f"; continue;
            case '\n': o += "\\n"; continue;
            case '\r': o += "\\r"; continue;
            case '\t': o += "\\t"; continue;
            default: break;
        }
        if (c < 0x20) {
            o += "\\u00";
            o.push_back(hex[c >> 4]);
            o.push_back(hex[c & 15]);
        } else if (c >= 0xD800 && c <= 0xDBFF && i + 1 < s.size() && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            uint32_t cp = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
            put_utf8(o, cp);
            i++;
        } else if (c >= 0xD800 && c <= 0xDFFF) {
            o += "\\u";
            o.push_back(hex[(c >> 12) & 15]);
            o.push_back(hex[(c >> 8) & 15]);
            o.push_back(hex[(c >> 4) & 15]);
            o.push_back(hex[c & 15]);
        } else {
            put_utf8(o, c);
        }
    }
    o.push_back('"');
}

inline void js_stringify(std::string& o, const JV& v) {
    switch (v.t) {
        case JV::Null: o += "null"; break;
        case JV::Bool: o += v.b ? "true" : "false"; break;
        case JV::Num: o += js_number(v.n); break;
        case JV::Str: js_quote(o, v.s); break;
        case JV::Arr: {
            o.push_back('[');
            for (size_t i = 0; i < v.a.size(); i++) {
                if (i) o.push_back(',');
                if (v.a[i]) js_stringify(o, *v.a[i]); else o += "null";
            }
            o.push_back(']');
            break;
        }
        case JV::Obj: {
            o.push_back('{');
            bool first = true;
            for (auto& k : v.o.keys()) {
                JVP e = v.o.get(k);
                if (!e) continue;  // undefined members are skipped
                if (!first) o.push_back(',');
                first = false;
                js_quote(o, k);
                o.push_back(':');
                js_stringify(o, *e);
            }
            o.push_back('}');
            break;
        }
    }
}

inline std::string stringify(const JV& v) { std::string o; js_stringify(o, v); return o; }

// ---- JSON.parse ------------------------------------------------------------------------------
struct Parser {
    const char* s;
    size_t n, i = 0;
    Parser(const char* s_, size_t n_) : s(s_), n(n_) {}
    [[noreturn]] void fail(const char* m) {
        throw std::runtime_error(std::string("JSON parse error: ") + m + " at " + std::to_string(i));
    }
    void ws() { while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++; }
    bool lit(const char* w) {
        size_t l = strlen(w);
        if (i + l <= n && memcmp(s + i, w, l) == 0) { i += l; return true; }
        return false;
    }
    u16s str() {
        if (s[i] != '"') fail("expected string");
        i++;
        u16s out;
        size_t start = i;
        while (true) {
            if (i >= n) fail("unterminated string");
            char c = s[i];
            if (c == '"') {
                break;
            } else if (c == '\\') {
                if (start < i) { u16s t = utf8_to_u16(s + start, i - start); out += t; }
                i++;
                char e = s[i++];
                switch (e) {
                    case '"': out.push_back(u'"'); break;
                    case '\\': out.push_back(u'\\'); break;
                    case '/': out.push_back(u'/'); break;
                    case 'b': out.push_back(u'\b'); break;
                    case 'f': out.push_back(u'\f'); break;
                    case 'n': out.push_back(u'\n'); break;
                    case 'r': out.push_back(u'\r'); break;
                    case 't': out.push_back(u'\t'); break;
                    case 'u': {
                        if (i + 4 > n) fail("bad \\u");
                        unsigned v = 0;
                        for (int k = 0; k < 4; k++) {
                            char h = s[i++];
                            v <<= 4;
                            if (h >= '0' && h <= '9') v |= h - '0';
                            else if (h >= 'a' && h <= 'f') v |= h - 'a' + 10;
                            else if (h >= 'A' && h <= 'F') v |= h - 'A' + 10;
                            else fail("bad hex");
                        }
                        out.push_back((char16_t)v);
                        break;
                    }
                    default: fail("bad escape");
                }
                start = i;
            } else {
                i++;
            }
        }
        if (start < i) { u16s t = utf8_to_u16(s + start, i - start); out += t; }
        i++;
        return out;
    }
    JVP value() {
        ws();
        if (i >= n) fail("eof");
        char c = s[i];
        if (c == '{') {
            i++;
            auto v = JV::obj();
            ws();
            if (s[i] == '}') { i++; return v; }
            while (true) {
                ws();
                u16s k = str();
                ws();
                if (s[i] != ':') fail("expected :");
                i++;
                JVP e = value();
                v->o.set(k, e);  // duplicate keys: value replaced, position kept (V8)
                ws();
                if (s[i] == ',') { i++; continue; }
                if (s[i] == '}') { i++; break; }
                fail("expected , or }");
            }
            return v;
        }
        if (c == '[') {
            i++;
            auto v = std::make_shared<JV>();
            v->t = JV::Arr;
            ws();
            if (s[i] == ']') { i++; return v; }
            while (true) {
                v->a.push_back(value());
                ws();
                if (s[i] == ',') { i++; continue; }
                if (s[i] == ']') { i++; break; }
                fail("expected , or ]");
            }
            return v;
        }
        if (c == '"') return JV::str(str());
        if (lit("true")) return JV::boolean(true);
        if (lit("false")) return JV::boolean(false);
        if (lit("null")) return JV::null();
        // number
        size_t st = i;
        if (s[i] == '-') i++;
        while (i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                         s[i] == '+' || s[i] == '-'))
            i++;
        if (st == i) fail("unexpected char");
        std::string num(s + st, i - st);
        return JV::num(strtod(num.c_str(), nullptr));
    }
};

inline JVP parse(const char* s, size_t n) {
    Parser p(s, n);
    JVP v = p.value();
    p.ws();
    if (p.i != n) p.fail("trailing data");
    return v;
}
inline JVP parse(const std::string& s) { return parse(s.data(), s.size()); }

// JS truthiness of an optional value (nullptr == undefined).
inline bool truthy(const JV* v) {
    if (!v) return false;
    switch (v->t) {
        case JV::Null: return false;
        case JV::Bool: return v->b;
        case JV::Num: return v->n != 0 && !std::isnan(v->n);
        case JV::Str: return !v->s.empty();
        default: return true;
    }
}

}  // namespace orc
