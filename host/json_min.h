// json_min.h — a small JSON reader for the host driver's sweep files (objects, arrays, numbers, strings,
// true/false/null). Numbers keep their integer value exactly when they are integers (int64 range).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace jmin {

struct Value {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    bool b = false;
    double num = 0.0;
    int64_t inum = 0;
    bool is_int = false;
    std::string str;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;

    const Value *get(const std::string &k) const
    {
        if (kind != Obj) return nullptr;
        auto it = obj.find(k);
        return it == obj.end() ? nullptr : &it->second;
    }
    int64_t as_int() const
    {
        if (kind == Bool) return b ? 1 : 0;
        if (kind != Num || !is_int) throw std::runtime_error("expected an integer");
        return inum;
    }
    bool as_bool() const
    {
        if (kind == Bool) return b;
        if (kind == Num && is_int) return inum != 0;
        throw std::runtime_error("expected a boolean");
    }
};

class Parser {
  public:
    explicit Parser(const std::string &s) : s_(s) {}
    Value parse()
    {
        Value v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

  private:
    const std::string &s_;
    size_t i_ = 0;
    [[noreturn]] void fail(const char *what) const
    {
        throw std::runtime_error(std::string("JSON: ") + what + " at offset " + std::to_string(i_));
    }
    void ws()
    {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
    }
    bool lit(const char *w)
    {
        size_t n = 0;
        while (w[n]) ++n;
        if (s_.compare(i_, n, w) != 0) return false;
        i_ += n;
        return true;
    }
    Value value()
    {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        Value v;
        const char c = s_[i_];
        if (c == '{') {
            v.kind = Value::Obj;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == '}') {
                ++i_;
                return v;
            }
            for (;;) {
                ws();
                if (i_ >= s_.size() || s_[i_] != '"') fail("expected a key");
                std::string k = string();
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
                ++i_;
                v.obj[k] = value();
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == '}') {
                    ++i_;
                    return v;
                }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = Value::Arr;
            ++i_;
            ws();
            if (i_ < s_.size() && s_[i_] == ']') {
                ++i_;
                return v;
            }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == ']') {
                    ++i_;
                    return v;
                }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.kind = Value::Str;
            v.str = string();
            return v;
        }
        if (lit("true")) {
            v.kind = Value::Bool;
            v.b = true;
            return v;
        }
        if (lit("false")) {
            v.kind = Value::Bool;
            return v;
        }
        if (lit("null")) return v;
        return number();
    }
    std::string string()
    {
        std::string out;
        ++i_;  // opening quote
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\') {
                if (i_ >= s_.size()) fail("bad escape");
                const char e = s_[i_++];
                c = e == 'n' ? '\n' : e == 't' ? '\t' : e == 'r' ? '\r' : e;
            }
            out.push_back(c);
        }
        if (i_ >= s_.size()) fail("unterminated string");
        ++i_;
        return out;
    }
    Value number()
    {
        Value v;
        v.kind = Value::Num;
        const size_t b = i_;
        if (i_ < s_.size() && (s_[i_] == '-' || s_[i_] == '+')) ++i_;
        bool integral = true;
        while (i_ < s_.size()) {
            const char c = s_[i_];
            if (c >= '0' && c <= '9') {
                ++i_;
            } else if (c == '.' || c == 'e' || c == 'E' || c == '-' || c == '+') {
                integral = false;
                ++i_;
            } else {
                break;
            }
        }
        if (b == i_) fail("unexpected character");
        const std::string t = s_.substr(b, i_ - b);
        v.num = std::strtod(t.c_str(), nullptr);
        if (integral) {
            v.is_int = true;
            v.inum = std::strtoll(t.c_str(), nullptr, 10);
        } else if (v.num == (double)(int64_t)v.num) {
            v.is_int = true;
            v.inum = (int64_t)v.num;
        }
        return v;
    }
};

}  // namespace jmin
