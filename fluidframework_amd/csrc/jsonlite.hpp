// jsonlite.hpp — host-side JSON for the engine's boundary: parsing ISequencedDocumentMessage logs
// and emitting SnapshotV1 bytes exactly as V8's JSON.stringify would (Node 12 / V8 7.8, which is
// what the reference's serializer runs on: merge-tree/src/test/testSerializer.ts:27-30).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mte {
namespace json {

// A parsed JSON value; objects keep member insertion order (duplicates replaced in place, V8).
struct Value {
    enum Kind : uint8_t { Null, False, True, Number, String, Array, Object } kind = Null;
    double num = 0;
    std::u16string str;
    std::vector<Value> items;                               // array elements
    std::vector<std::pair<std::u16string, Value>> members;  // object members
    const Value* get(const char16_t* k) const {
        for (auto& m : members)
            if (m.first == k) return &m.second;
        return nullptr;
    }
};

inline void append_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
        o.push_back((char)cp);
    } else if (cp < 0x800) {
        o.push_back((char)(0xC0 | (cp >> 6)));
        o.push_back((char)(0x80 | (cp & 63)));
    } else if (cp < 0x10000) {
        o.push_back((char)(0xE0 | (cp >> 12)));
        o.push_back((char)(0x80 | ((cp >> 6) & 63)));
        o.push_back((char)(0x80 | (cp & 63)));
    } else {
        o.push_back((char)(0xF0 | (cp >> 18)));
        o.push_back((char)(0x80 | ((cp >> 12) & 63)));
        o.push_back((char)(0x80 | ((cp >> 6) & 63)));
        o.push_back((char)(0x80 | (cp & 63)));
    }
}

inline void decode_utf8(const char* s, size_t n, std::u16string& out) {
    for (size_t i = 0; i < n;) {
        uint8_t c = (uint8_t)s[i];
        uint32_t cp;
        size_t k;
        if (c < 0x80) { cp = c; k = 1; }
        else if (c < 0xE0) { cp = c & 31; k = 2; }
        else if (c < 0xF0) { cp = c & 15; k = 3; }
        else { cp = c & 7; k = 4; }
        for (size_t j = 1; j < k && i + j < n; j++) cp = (cp << 6) | ((uint8_t)s[i + j] & 63);
        i += k;
        if (cp >= 0x10000) {
            cp -= 0x10000;
            out.push_back((char16_t)(0xD800 | (cp >> 10)));
            out.push_back((char16_t)(0xDC00 | (cp & 1023)));
        } else {
            out.push_back((char16_t)cp);
        }
    }
}

// UTF-16 -> UTF-8, lone surrogates as U+FFFD (Buffer.from(string) semantics).
inline std::string to_utf8(const char16_t* s, size_t n) {
    std::string o;
    o.reserve(n);
    for (size_t i = 0; i < n; i++) {
        uint32_t c = s[i];
        if (c >= 0xD800 && c < 0xDC00 && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] < 0xE000) {
            append_utf8(o, 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00));
            i++;
        } else if (c >= 0xD800 && c < 0xE000) {
            append_utf8(o, 0xFFFD);
        } else {
            append_utf8(o, c);
        }
    }
    return o;
}

// JSON.stringify(string): escapes per ES2019 well-formed stringify.
inline void quote(std::string& o, const char16_t* s, size_t n) {
    static const char hx[] = "0123456789abcdef";
    o.push_back('"');
    for (size_t i = 0; i < n; i++) {
        uint32_t c = s[i];
        if (c == '"') { o += "\\\""; continue; }
        if (c == '\\') { o += "\\\\"; continue; }
        if (c < 0x20) {
            switch (c) {
                case '\b': o += "\\b"; break;
                case '\f': o += "\\f"; break;
                case '\n': o += "\\n"; break;
                case '\r': o += "\\r"; break;
                case '\t': o += "\\t"; break;
                default: o += "\\u00"; o.push_back(hx[c >> 4]); o.push_back(hx[c & 15]);
            }
            continue;
        }
        if (c >= 0xD800 && c < 0xE000) {
            if (c < 0xDC00 && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] < 0xE000) {
                append_utf8(o, 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00));
                i++;
            } else {
                o += "\\u";
                o.push_back(hx[(c >> 12) & 15]);
                o.push_back(hx[(c >> 8) & 15]);
                o.push_back(hx[(c >> 4) & 15]);
                o.push_back(hx[c & 15]);
            }
            continue;
        }
        append_utf8(o, c);
    }
    o.push_back('"');
}
inline void quote(std::string& o, const std::u16string& s) { quote(o, s.data(), s.size()); }

// Number::toString (ECMA-262 7.1.12.1): shortest round-trip digits, JS exponent rules.
inline std::string number(double x) {
    if (!std::isfinite(x)) return "null";
    if (x == 0) return "0";
    char buf[40];
    std::string sign = x < 0 ? "-" : "";
    double a = std::fabs(x);
    int prec = 1;
    for (; prec <= 17; prec++) {
        snprintf(buf, sizeof buf, "%.*e", prec - 1, a);
        if (strtod(buf, nullptr) == a) break;
    }
    char* e = strchr(buf, 'e');
    int exp10 = atoi(e + 1);
    std::string dig;
    for (char* q = buf; q < e; q++)
        if (*q >= '0' && *q <= '9') dig.push_back(*q);
    while (dig.size() > 1 && dig.back() == '0') dig.pop_back();
    const int k = (int)dig.size(), n = exp10 + 1;
    std::string r;
    if (k <= n && n <= 21) r = dig + std::string(n - k, '0');
    else if (n > 0 && n <= 21) r = dig.substr(0, n) + "." + dig.substr(n);
    else if (n > -6 && n <= 0) r = "0." + std::string(-n, '0') + dig;
    else {
        r = dig.substr(0, 1) + (k > 1 ? "." + dig.substr(1) : "") + "e" + (n - 1 < 0 ? "-" : "+") +
            std::to_string(std::abs(n - 1));
    }
    return sign + r;
}

// Canonical array-index key ("0".."4294967294"): JS enumerates these first, ascending.
inline bool array_index(const std::u16string& k, uint32_t* v) {
    if (k.empty() || k.size() > 10 || (k.size() > 1 && k[0] == u'0')) return false;
    uint64_t x = 0;
    for (char16_t c : k) {
        if (c < u'0' || c > u'9') return false;
        x = x * 10 + (uint64_t)(c - u'0');
    }
    if (x > 4294967294ull) return false;
    *v = (uint32_t)x;
    return true;
}

// Object.keys order of an object value's members.
inline std::vector<size_t> key_order(const Value& v) {
    std::vector<std::pair<uint32_t, size_t>> idx;
    std::vector<size_t> rest;
    for (size_t i = 0; i < v.members.size(); i++) {
        uint32_t a;
        if (array_index(v.members[i].first, &a)) idx.emplace_back(a, i);
        else rest.push_back(i);
    }
    std::sort(idx.begin(), idx.end());
    std::vector<size_t> out;
    for (auto& p : idx) out.push_back(p.second);
    out.insert(out.end(), rest.begin(), rest.end());
    return out;
}

inline void stringify(std::string& o, const Value& v) {
    switch (v.kind) {
        case Value::Null: o += "null"; break;
        case Value::False: o += "false"; break;
        case Value::True: o += "true"; break;
        case Value::Number: o += number(v.num); break;
        case Value::String: quote(o, v.str); break;
        case Value::Array:
            o.push_back('[');
            for (size_t i = 0; i < v.items.size(); i++) {
                if (i) o.push_back(',');
                stringify(o, v.items[i]);
            }
            o.push_back(']');
            break;
        case Value::Object: {
            o.push_back('{');
            bool first = true;
            for (size_t i : key_order(v)) {
                if (!first) o.push_back(',');
                first = false;
                quote(o, v.members[i].first);
                o.push_back(':');
                stringify(o, v.members[i].second);
            }
            o.push_back('}');
            break;
        }
    }
}
inline std::string stringify(const Value& v) {
    std::string o;
    stringify(o, v);
    return o;
}

class Reader {
   public:
    Reader(const char* p, size_t n) : p_(p), n_(n) {}
    Value parse_document() {
        Value v = value();
        skip();
        if (i_ != n_) error("trailing characters");
        return v;
    }

   private:
    const char* p_;
    size_t n_, i_ = 0;
    [[noreturn]] void error(const char* what) {
        throw std::runtime_error(std::string("op-log JSON: ") + what + " at byte " + std::to_string(i_));
    }
    void skip() {
        while (i_ < n_ && (p_[i_] == ' ' || p_[i_] == '\n' || p_[i_] == '\r' || p_[i_] == '\t')) i_++;
    }
    bool eat(const char* w) {
        size_t k = strlen(w);
        if (n_ - i_ >= k && !memcmp(p_ + i_, w, k)) {
            i_ += k;
            return true;
        }
        return false;
    }
    std::u16string string() {
        std::u16string s;
        i_++;  // opening quote
        size_t run = i_;
        for (;;) {
            if (i_ >= n_) error("unterminated string");
            char c = p_[i_];
            if (c == '"') break;
            if (c != '\\') {
                i_++;
                continue;
            }
            decode_utf8(p_ + run, i_ - run, s);
            if (i_ + 1 >= n_) error("bad escape");
            char e = p_[i_ + 1];
            i_ += 2;
            switch (e) {
                case '"': s.push_back(u'"'); break;
                case '\\': s.push_back(u'\\'); break;
                case '/': s.push_back(u'/'); break;
                case 'b': s.push_back(u'\b'); break;
                case 'f': s.push_back(u'\f'); break;
                case 'n': s.push_back(u'\n'); break;
                case 'r': s.push_back(u'\r'); break;
                case 't': s.push_back(u'\t'); break;
                case 'u': {
                    if (n_ - i_ < 4) error("bad \\u escape");
                    uint32_t cu = 0;
                    for (int k = 0; k < 4; k++) {
                        char h = p_[i_++];
                        int d = (h >= '0' && h <= '9') ? h - '0' : (h >= 'a' && h <= 'f') ? h - 'a' + 10
                                : (h >= 'A' && h <= 'F') ? h - 'A' + 10 : -1;
                        if (d < 0) error("bad hex digit");
                        cu = cu * 16 + (uint32_t)d;
                    }
                    s.push_back((char16_t)cu);
                    break;
                }
                default: error("bad escape");
            }
            run = i_;
        }
        decode_utf8(p_ + run, i_ - run, s);
        i_++;
        return s;
    }
    Value value() {
        skip();
        if (i_ >= n_) error("unexpected end");
        Value v;
        char c = p_[i_];
        if (c == '"') {
            v.kind = Value::String;
            v.str = string();
        } else if (c == '{') {
            v.kind = Value::Object;
            i_++;
            skip();
            if (i_ < n_ && p_[i_] == '}') {
                i_++;
                return v;
            }
            for (;;) {
                skip();
                if (i_ >= n_ || p_[i_] != '"') error("expected member name");
                std::u16string k = string();
                skip();
                if (i_ >= n_ || p_[i_] != ':') error("expected ':'");
                i_++;
                Value m = value();
                bool dup = false;
                for (auto& e : v.members)
                    if (e.first == k) {
                        e.second = std::move(m);
                        dup = true;
                        break;
                    }
                if (!dup) v.members.emplace_back(std::move(k), std::move(m));
                skip();
                if (i_ < n_ && p_[i_] == ',') { i_++; continue; }
                if (i_ < n_ && p_[i_] == '}') { i_++; break; }
                error("expected ',' or '}'");
            }
        } else if (c == '[') {
            v.kind = Value::Array;
            i_++;
            skip();
            if (i_ < n_ && p_[i_] == ']') {
                i_++;
                return v;
            }
            for (;;) {
                v.items.push_back(value());
                skip();
                if (i_ < n_ && p_[i_] == ',') { i_++; continue; }
                if (i_ < n_ && p_[i_] == ']') { i_++; break; }
                error("expected ',' or ']'");
            }
        } else if (eat("true")) {
            v.kind = Value::True;
        } else if (eat("false")) {
            v.kind = Value::False;
        } else if (eat("null")) {
            v.kind = Value::Null;
        } else {
            size_t st = i_;
            while (i_ < n_ && strchr("+-0123456789.eE", p_[i_])) i_++;
            if (st == i_) error("unexpected character");
            v.kind = Value::Number;
            v.num = strtod(std::string(p_ + st, i_ - st).c_str(), nullptr);
        }
        return v;
    }
};

inline Value parse(const char* p, size_t n) { return Reader(p, n).parse_document(); }

// ---- JavaScript semantics used by matchProperties (properties.ts:62-93) ----------------------
inline bool truthy(const Value* v) {
    if (!v) return false;
    switch (v->kind) {
        case Value::Null: case Value::False: return false;
        case Value::Number: return v->num != 0 && !std::isnan(v->num);
        case Value::String: return !v->str.empty();
        default: return true;
    }
}
inline std::vector<std::u16string> for_in(const Value* v) {
    std::vector<std::u16string> k;
    if (!v) return k;
    if (v->kind == Value::Object) {
        for (size_t i : key_order(*v)) k.push_back(v->members[i].first);
    } else if (v->kind == Value::Array || v->kind == Value::String) {
        size_t n = v->kind == Value::Array ? v->items.size() : v->str.size();
        for (size_t i = 0; i < n; i++) {
            std::string d = std::to_string(i);
            k.emplace_back(d.begin(), d.end());
        }
    }
    return k;
}
// v[key] for object / array / string receivers; `tmp` holds a synthesized one-char string.
inline const Value* member(const Value* v, const std::u16string& key, Value& tmp) {
    if (!v) return nullptr;
    if (v->kind == Value::Object) {
        for (auto& m : v->members)
            if (m.first == key) return &m.second;
        return nullptr;
    }
    uint32_t i;
    if (!array_index(key, &i)) return nullptr;
    if (v->kind == Value::Array) return i < v->items.size() ? &v->items[i] : nullptr;
    if (v->kind == Value::String && i < v->str.size()) {
        tmp.kind = Value::String;
        tmp.str = std::u16string(1, v->str[i]);
        return &tmp;
    }
    return nullptr;
}
inline bool is_object_typed(const Value* v) {  // typeof v === "object"
    return v && (v->kind == Value::Object || v->kind == Value::Array || v->kind == Value::Null);
}
inline bool strictly_equal_primitive(const Value* a, const Value* b) {
    if (!a || !b) return a == b;
    if (a->kind != b->kind) return false;
    if (a->kind == Value::Number) return a->num == b->num;
    if (a->kind == Value::String) return a->str == b->str;
    return a->kind == Value::Null || a->kind == Value::True || a->kind == Value::False;
}
inline bool match_properties(const Value* a, const Value* b) {
    if (truthy(a)) {
        if (!truthy(b)) return false;
        for (auto& k : for_in(a)) {
            Value ta, tb;
            const Value* bk = member(b, k, tb);
            const Value* ak = member(a, k, ta);
            if (!bk) return false;
            if (is_object_typed(bk)) {
                if (!match_properties(ak, bk)) return false;
            } else if (!strictly_equal_primitive(bk, ak)) {
                return false;
            }
        }
        for (auto& k : for_in(b)) {
            Value ta;
            if (!member(a, k, ta)) return false;
        }
        return true;
    }
    return !truthy(b);
}

}  // namespace json
}  // namespace mte
