// json.cpp — korali::Json (see json.hpp).
#include "json.hpp"

#include <atomic>
#include <mutex>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>

namespace korali {

struct Json::Packed {
  std::vector<double> d;
  std::atomic<std::vector<Json> *> nodes{nullptr};  // built by a const reader, then immutable
  explicit Packed(std::vector<double> &&v) : d(std::move(v)) {}
  ~Packed() { delete nodes.load(); }
};


namespace {
// never destroyed: entries may hold Python callables, which must not be
// released after the interpreter has finalised.  A deque: references handed
// out by getFunction stay valid while other threads register functions.
std::deque<Function> &functionTable() {
  static auto *t = new std::deque<Function>();
  return *t;
}
std::mutex &functionMutex() {
  static std::mutex m;
  return m;
}
const char *typeName(Json::Type t) {
  switch (t) {
    case Json::Type::Null: return "null";
    case Json::Type::Bool: return "boolean";
    case Json::Type::Int:
    case Json::Type::UInt:
    case Json::Type::Double: return "number";
    case Json::Type::String: return "string";
    case Json::Type::Array: return "array";
    case Json::Type::Object: return "object";
  }
  return "?";
}
}  // namespace

size_t registerFunction(Function f) {
  std::lock_guard<std::mutex> g(functionMutex());
  functionTable().push_back(std::move(f));
  return functionTable().size() - 1;
}

Function &getFunction(size_t index) {
  std::lock_guard<std::mutex> g(functionMutex());
  if (index >= functionTable().size()) throw std::runtime_error("invalid function index " + std::to_string(index));
  return functionTable()[index];
}

Json::Json(void (*fn)(Sample &)) : t_(Type::UInt) { v_.u = registerFunction(Function(fn)); }

void Json::release() noexcept {
  switch (t_) {
    case Type::String: delete v_.s; break;
    case Type::Array:
      if (packed_)
        delete v_.pk;
      else
        delete v_.a;
      break;
    case Type::Object: delete v_.o; break;
    default: break;
  }
  t_ = Type::Null;
  packed_ = false;
  v_.u = 0;
}

void Json::copyFrom(const Json &o) {
  switch (o.t_) {
    case Type::String: v_.s = new std::string(*o.v_.s); break;
    case Type::Array:
      if (o.packed_)
        v_.pk = makePacked(std::vector<double>(o.v_.pk->d));
      else
        v_.a = new std::vector<Json>(*o.v_.a);
      break;
    case Type::Object: v_.o = new std::map<std::string, Json>(*o.v_.o); break;
    default: v_ = o.v_;
  }
}


Json::Packed *Json::makePacked(std::vector<double> &&v) { return new Packed(std::move(v)); }

size_t Json::size() const {
  return t_ == Type::Array ? (packed_ ? v_.pk->d.size() : v_.a->size()) : t_ == Type::Object ? v_.o->size() : 0;
}

const std::vector<double> *Json::packedDoubles() const { return t_ == Type::Array && packed_ ? &v_.pk->d : nullptr; }

void Json::unpack() {
  if (!packed_) return;
  std::vector<Json> *a = v_.pk->nodes.exchange(nullptr);
  if (!a) a = new std::vector<Json>(v_.pk->d.begin(), v_.pk->d.end());
  delete v_.pk;
  v_.a = a;
  packed_ = false;
}

const std::vector<Json> &Json::constNodes() const {
  if (!packed_) return *v_.a;
  std::vector<Json> *n = v_.pk->nodes.load(std::memory_order_acquire);
  if (n) return *n;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  n = v_.pk->nodes.load(std::memory_order_relaxed);
  if (!n) {
    n = new std::vector<Json>(v_.pk->d.begin(), v_.pk->d.end());
    v_.pk->nodes.store(n, std::memory_order_release);
  }
  return *n;
}

std::vector<Json> &Json::arrayRef() {
  if (t_ == Type::Null) *this = array();
  if (t_ != Type::Array) throw std::runtime_error("push_back on a non-array JSON value");
  unpack();
  return *v_.a;
}

const std::map<std::string, Json> &Json::items() const {
  static const std::map<std::string, Json> none;
  return t_ == Type::Object ? *v_.o : none;
}

const std::vector<Json> &Json::elements() const {
  static const std::vector<Json> none;
  if (t_ != Type::Array) return none;
  return constNodes();
}

Json &Json::operator[](const std::string &key) {
  if (t_ == Type::Null) *this = object();
  if (t_ != Type::Object)
    throw std::runtime_error("cannot index a JSON " + std::string(typeName(t_)) + " with key '" + key + "'");
  return (*v_.o)[key];
}

Json &Json::operator[](size_t idx) {
  if (t_ == Type::Null) *this = array();
  if (t_ != Type::Array)
    throw std::runtime_error("cannot index a JSON " + std::string(typeName(t_)) + " with [" + std::to_string(idx) + "]");
  unpack();
  if (idx >= v_.a->size()) v_.a->resize(idx + 1);
  return (*v_.a)[idx];
}

const Json &Json::at(const std::string &key) const {
  if (t_ != Type::Object) throw std::runtime_error("missing key '" + key + "'");
  const auto it = v_.o->find(key);
  if (it == v_.o->end()) throw std::runtime_error("missing key '" + key + "'");
  return it->second;
}

const Json &Json::at(size_t idx) const {
  if (t_ != Type::Array || idx >= size()) throw std::runtime_error("index out of range");
  return constNodes()[idx];
}

double Json::getDouble() const {
  switch (t_) {
    case Type::Double: return v_.d;
    case Type::Int: return (double)v_.i;
    case Type::UInt: return (double)v_.u;
    case Type::Bool: return v_.b ? 1.0 : 0.0;
    default: throw std::runtime_error(std::string("expected a number, found a ") + typeName(t_));
  }
}

long long Json::getInt() const {
  switch (t_) {
    case Type::Int: return v_.i;
    case Type::UInt: return (long long)v_.u;
    case Type::Double:
      if (v_.d != std::floor(v_.d)) throw std::runtime_error("expected an integer, found " + std::to_string(v_.d));
      return (long long)v_.d;
    case Type::Bool: return v_.b ? 1 : 0;
    default: throw std::runtime_error(std::string("expected an integer, found a ") + typeName(t_));
  }
}

unsigned long long Json::getUInt() const {
  switch (t_) {
    case Type::UInt: return v_.u;
    case Type::Int:
      if (v_.i < 0) throw std::runtime_error("expected a non-negative integer, found " + std::to_string(v_.i));
      return (unsigned long long)v_.i;
    case Type::Double:
      if (!(v_.d >= 0) || v_.d != std::floor(v_.d))
        throw std::runtime_error("expected a non-negative integer, found " + std::to_string(v_.d));
      return v_.d >= 1.8446744073709552e19 ? ~0ULL : (unsigned long long)v_.d;
    case Type::Bool: return v_.b ? 1 : 0;
    default: throw std::runtime_error(std::string("expected an integer, found a ") + typeName(t_));
  }
}

bool Json::getBool() const {
  if (t_ == Type::Bool) return v_.b;
  if (t_ == Type::Int) return v_.i != 0;
  if (t_ == Type::UInt) return v_.u != 0;
  throw std::runtime_error(std::string("expected a boolean, found a ") + typeName(t_));
}

const std::string &Json::getString() const {
  if (t_ != Type::String) throw std::runtime_error(std::string("expected a string, found a ") + typeName(t_));
  return *v_.s;
}

std::vector<double> Json::getDoubleVector() const {
  if (t_ != Type::Array) throw std::runtime_error(std::string("expected an array, found a ") + typeName(t_));
  if (packed_) return v_.pk->d;
  std::vector<double> v;
  v.reserve(v_.a->size());
  for (const auto &x : *v_.a) v.push_back(x.getDouble());
  return v;
}

// ----------------------------------------------------------------- dump
namespace {
void dumpString(std::string &out, const std::string &s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\t': out += "\\t"; break;
      case '\r': out += "\\r"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof(b), "\\u%04x", c);
          out += b;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}
void dumpDouble(std::string &out, double d) {
  if (std::isnan(d)) {
    out += "NaN";
  } else if (std::isinf(d)) {
    out += d > 0 ? "Infinity" : "-Infinity";
  } else {
    // shortest text that reads back to the same double (nlohmann's grisu2
    // output has the same property)
    char b[32];
    const auto r = std::to_chars(b, b + sizeof(b), d);
    out.append(b, r.ptr);
    if (std::find_if(b, r.ptr, [](char c) { return c == '.' || c == 'e' || c == 'E'; }) == r.ptr) out += ".0";
  }
}
}  // namespace

void Json::dumpTo(std::string &out, int indent, int level) const {
  auto nl = [&](int l) {
    if (indent < 0) return;
    out += '\n';
    out.append((size_t)(indent * l), ' ');
  };
  switch (t_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += v_.b ? "true" : "false"; break;
    case Type::Int: out += std::to_string(v_.i); break;
    case Type::UInt: out += std::to_string(v_.u); break;
    case Type::Double: dumpDouble(out, v_.d); break;
    case Type::String: dumpString(out, *v_.s); break;
    case Type::Array: {
      out += '[';
      if (packed_) {
        for (size_t k = 0; k < v_.pk->d.size(); k++) {
          if (k) out += ',';
          nl(level + 1);
          dumpDouble(out, v_.pk->d[k]);
        }
        if (!v_.pk->d.empty()) nl(level);
        out += ']';
        break;
      }
      bool first = true;
      for (const auto &x : *v_.a) {
        if (!first) out += ',';
        first = false;
        nl(level + 1);
        x.dumpTo(out, indent, level + 1);
      }
      if (!v_.a->empty()) nl(level);
      out += ']';
      break;
    }
    case Type::Object: {
      out += '{';
      bool first = true;
      for (const auto &kv : *v_.o) {
        if (!first) out += ',';
        first = false;
        nl(level + 1);
        dumpString(out, kv.first);
        out += indent < 0 ? ":" : ": ";
        kv.second.dumpTo(out, indent, level + 1);
      }
      if (!v_.o->empty()) nl(level);
      out += '}';
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dumpTo(out, indent, 0);
  return out;
}

// ---------------------------------------------------------------- parse
namespace {
struct Parser {
  const std::string &s;
  size_t p = 0;
  [[noreturn]] void fail(const std::string &m) {
    throw std::runtime_error("JSON parse error at offset " + std::to_string(p) + ": " + m);
  }
  void ws() {
    while (p < s.size() && (s[p] == ' ' || s[p] == '\n' || s[p] == '\t' || s[p] == '\r')) p++;
  }
  bool lit(const char *w) {
    const size_t n = strlen(w);
    if (s.compare(p, n, w) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  Json value() {
    ws();
    if (p >= s.size()) fail("unexpected end");
    const char c = s[p];
    if (c == '{') {
      p++;
      Json o = Json::object();
      ws();
      if (p < s.size() && s[p] == '}') {
        p++;
        return o;
      }
      for (;;) {
        ws();
        if (p >= s.size() || s[p] != '"') fail("expected a key");
        const std::string k = str();
        ws();
        if (p >= s.size() || s[p] != ':') fail("expected ':'");
        p++;
        o[k] = value();
        ws();
        if (p < s.size() && s[p] == ',') {
          p++;
          continue;
        }
        if (p < s.size() && s[p] == '}') {
          p++;
          return o;
        }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      p++;
      Json a = Json::array();
      ws();
      if (p < s.size() && s[p] == ']') {
        p++;
        return a;
      }
      for (;;) {
        a.push_back(value());
        ws();
        if (p < s.size() && s[p] == ',') {
          p++;
          continue;
        }
        if (p < s.size() && s[p] == ']') {
          p++;
          return a;
        }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') return Json(str());
    if (lit("true")) return Json(true);
    if (lit("false")) return Json(false);
    if (lit("null")) return Json();
    if (lit("NaN")) return Json(std::nan(""));
    if (lit("Infinity")) return Json(INFINITY);
    if (lit("-Infinity")) return Json(-INFINITY);
    return number();
  }
  std::string str() {
    std::string r;
    p++;  // opening quote
    while (p < s.size() && s[p] != '"') {
      char c = s[p++];
      if (c == '\\') {
        if (p >= s.size()) fail("bad escape");
        const char e = s[p++];
        switch (e) {
          case 'n': r += '\n'; break;
          case 't': r += '\t'; break;
          case 'r': r += '\r'; break;
          case 'b': r += '\b'; break;
          case 'f': r += '\f'; break;
          case 'u': {
            if (p + 4 > s.size()) fail("bad \\u escape");
            const unsigned cp = (unsigned)std::stoul(s.substr(p, 4), nullptr, 16);
            p += 4;
            if (cp < 0x80) {
              r += (char)cp;
            } else if (cp < 0x800) {
              r += (char)(0xC0 | (cp >> 6));
              r += (char)(0x80 | (cp & 0x3F));
            } else {
              r += (char)(0xE0 | (cp >> 12));
              r += (char)(0x80 | ((cp >> 6) & 0x3F));
              r += (char)(0x80 | (cp & 0x3F));
            }
            break;
          }
          default: r += e;
        }
      } else {
        r += c;
      }
    }
    if (p >= s.size()) fail("unterminated string");
    p++;
    return r;
  }
  Json number() {
    const size_t b = p;
    if (p < s.size() && (s[p] == '-' || s[p] == '+')) p++;
    bool isFloat = false;
    while (p < s.size() && (isdigit((unsigned char)s[p]) || s[p] == '.' || s[p] == 'e' || s[p] == 'E' ||
                            ((s[p] == '-' || s[p] == '+') && (s[p - 1] == 'e' || s[p - 1] == 'E')))) {
      if (s[p] == '.' || s[p] == 'e' || s[p] == 'E') isFloat = true;
      p++;
    }
    if (p == b) fail("unexpected character");
    const std::string t = s.substr(b, p - b);
    if (!isFloat) {
      errno = 0;
      if (t[0] == '-') {
        const long long v = strtoll(t.c_str(), nullptr, 10);
        if (errno == 0) return Json(v);
      } else {
        const unsigned long long v = strtoull(t.c_str(), nullptr, 10);
        if (errno == 0) return Json(v);
      }
    }
    return Json(strtod(t.c_str(), nullptr));
  }
};
}  // namespace

Json Json::parse(const std::string &text) {
  Parser ps{text};
  Json v = ps.value();
  ps.ws();
  if (ps.p != text.size()) ps.fail("trailing characters");
  return v;
}

}  // namespace korali
