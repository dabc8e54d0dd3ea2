// json.hpp — the JSON value behind korali::Experiment / korali::Sample.
//
// Korali keeps every experiment setting and every piece of solver state in
// one JSON tree (knlohmann::json in the reference, source/auxiliar/
// koraliJson.hpp).  This is a small self-contained equivalent with the
// behaviour the API relies on: operator[] auto-vivifies objects and
// extends arrays, integers keep 64 bits (random seeds), doubles round-trip
// exactly (17 significant digits) and non-finite numbers are written and
// read as Infinity / -Infinity / NaN like the reference's result files.
// Functions are stored as an index into the process-wide function table
// (the reference's _functionVector, py2json.hpp:54-58).
#pragma once

#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace korali {

class Sample;
using Function = std::function<void(Sample &)>;

// process-wide table of user functions; JSON stores their index
size_t registerFunction(Function f);
Function &getFunction(size_t index);

class Json {
 public:
  enum class Type { Null, Bool, Int, UInt, Double, String, Array, Object };

  Json() { v_.u = 0; }
  Json(std::nullptr_t) { v_.u = 0; }
  Json(bool b) : t_(Type::Bool) { v_.u = 0, v_.b = b; }
  Json(int v) : t_(Type::Int) { v_.i = v; }
  Json(long v) : t_(Type::Int) { v_.i = v; }
  Json(long long v) : t_(Type::Int) { v_.i = v; }
  Json(unsigned v) : t_(Type::UInt) { v_.u = v; }
  Json(unsigned long v) : t_(Type::UInt) { v_.u = v; }
  Json(unsigned long long v) : t_(Type::UInt) { v_.u = v; }
  Json(double v) : t_(Type::Double) { v_.d = v; }
  Json(float v) : t_(Type::Double) { v_.d = v; }
  Json(const char *s) : t_(Type::String) { v_.s = new std::string(s); }
  Json(const std::string &s) : t_(Type::String) { v_.s = new std::string(s); }
  Json(void (*fn)(Sample &));  // registers the function, stores its index
  // an array of doubles is held packed (one contiguous block, no per-element
  // node) until an element is addressed as a node (operator[], at,
  // elements(), push_back): vectors and matrices of solver state, the bulk of
  // every result file, are built, copied, read back and dumped as blocks
  template <typename T>
  Json(const std::vector<T> &v) : t_(Type::Array) {
    if constexpr (std::is_same<T, double>::value || std::is_same<T, float>::value) {
      packed_ = true;
      v_.pk = makePacked(std::vector<double>(v.begin(), v.end()));
    } else {
      v_.a = new std::vector<Json>();
      v_.a->reserve(v.size());
      for (const auto &x : v) v_.a->emplace_back(x);
    }
  }
  Json(std::vector<double> &&v) : t_(Type::Array), packed_(true) { v_.pk = makePacked(std::move(v)); }
  Json(const Json &o) : t_(o.t_), packed_(o.packed_) { copyFrom(o); }
  Json(Json &&o) noexcept : t_(o.t_), packed_(o.packed_), v_(o.v_) {
    o.t_ = Type::Null;
    o.packed_ = false;
    o.v_.u = 0;
  }
  Json &operator=(const Json &o) {
    if (this != &o) {
      Json c(o);
      swap(c);
    }
    return *this;
  }
  Json &operator=(Json &&o) noexcept {
    if (this != &o) {
      Json c(std::move(o));
      swap(c);
    }
    return *this;
  }
  ~Json() { release(); }
  void swap(Json &o) noexcept {
    std::swap(t_, o.t_);
    std::swap(packed_, o.packed_);
    std::swap(v_, o.v_);
  }

  static Json array() {
    Json j;
    j.t_ = Type::Array;
    j.v_.a = new std::vector<Json>();
    return j;
  }
  static Json object() {
    Json j;
    j.t_ = Type::Object;
    j.v_.o = new std::map<std::string, Json>();
    return j;
  }
  static Json parse(const std::string &text);

  Type type() const { return t_; }
  bool is_null() const { return t_ == Type::Null; }
  bool is_bool() const { return t_ == Type::Bool; }
  bool is_number() const { return t_ == Type::Int || t_ == Type::UInt || t_ == Type::Double; }
  bool is_integer() const { return t_ == Type::Int || t_ == Type::UInt; }
  bool is_string() const { return t_ == Type::String; }
  bool is_array() const { return t_ == Type::Array; }
  bool is_object() const { return t_ == Type::Object; }

  // auto-vivifying access (null becomes object / array)
  Json &operator[](const std::string &key);
  Json &operator[](const char *key) { return (*this)[std::string(key)]; }
  Json &operator[](size_t idx);
  Json &operator[](int idx) { return (*this)[(size_t)idx]; }
  const Json &at(const std::string &key) const;
  const Json &at(size_t idx) const;
  bool contains(const std::string &key) const { return t_ == Type::Object && v_.o->count(key) != 0; }
  void erase(const std::string &key) {
    if (t_ == Type::Object) v_.o->erase(key);
  }
  size_t size() const;
  void push_back(const Json &v) { arrayRef().push_back(v); }
  void push_back(Json &&v) { arrayRef().push_back(std::move(v)); }
  // the packed doubles of an array held packed, else nullptr (fast paths of
  // readers that need no nodes)
  const std::vector<double> *packedDoubles() const;
  const std::map<std::string, Json> &items() const;
  const std::vector<Json> &elements() const;

  double getDouble() const;
  long long getInt() const;
  unsigned long long getUInt() const;
  bool getBool() const;
  const std::string &getString() const;
  std::vector<double> getDoubleVector() const;
  template <typename T>
  T get() const;

  // implicit conversion to a value type, as knlohmann::json allows
  // (examples/features/running.cxx/_model/direct.hpp:8:
  //  `float x = k["Parameters"][0];`, `std::vector<double> p = s["Parameters"];`)
  template <typename T, typename = typename std::enable_if<!std::is_pointer<T>::value &&
                                                           !std::is_same<T, Json>::value>::type>
  operator T() const {
    return get<T>();
  }
  // comparisons with plain values (sample.cpp: `(*_self)["Module"] == "Solver"`)
  bool operator==(const char *v) const { return is_string() && *v_.s == v; }
  bool operator==(const std::string &v) const { return is_string() && *v_.s == v; }
  bool operator==(bool v) const { return is_bool() && v_.b == v; }
  bool operator==(double v) const { return is_number() && getDouble() == v; }
  bool operator==(int v) const { return is_number() && getDouble() == (double)v; }
  template <typename T>
  bool operator!=(const T &v) const {
    return !(*this == v);
  }

  std::string dump(int indent = -1) const;

 private:
  // 16 bytes a node: the tag and one word (a scalar, or the heap-held
  // string / array / object) -- result files hold 10^5-10^6 numbers
  // (Sample Population, databases), built and copied every save.  packed_:
  // an Array held as doubles (pk) rather than nodes (a).  A const reader that
  // needs nodes (at(i), elements()) gets them built once beside the doubles
  // under a lock and published atomically -- const reads never change the
  // representation, so several threads may read one Json (the Concurrent
  // conduit's workers); a non-const access converts to nodes.
  struct Packed;
  static Packed *makePacked(std::vector<double> &&v);
  Type t_ = Type::Null;
  bool packed_ = false;
  union {
    bool b;
    long long i;
    unsigned long long u;
    double d;
    std::string *s;
    std::vector<Json> *a;
    Packed *pk;
    std::map<std::string, Json> *o;
  } v_;
  void unpack();                                // packed -> nodes (non-const paths)
  const std::vector<Json> &constNodes() const;  // the nodes of an array, packed or not
  void release() noexcept;
  void copyFrom(const Json &o);
  std::vector<Json> &arrayRef();  // null becomes an empty array
  void dumpTo(std::string &out, int indent, int level) const;
};

template <>
inline double Json::get<double>() const { return getDouble(); }
template <>
inline float Json::get<float>() const { return (float)getDouble(); }
template <>
inline int Json::get<int>() const { return (int)getInt(); }
template <>
inline long Json::get<long>() const { return (long)getInt(); }
template <>
inline size_t Json::get<size_t>() const { return (size_t)getUInt(); }
template <>
inline bool Json::get<bool>() const { return getBool(); }
template <>
inline std::string Json::get<std::string>() const { return getString(); }
template <>
inline std::vector<double> Json::get<std::vector<double>>() const { return getDoubleVector(); }
template <>
inline long long Json::get<long long>() const { return getInt(); }
template <>
inline unsigned Json::get<unsigned>() const { return (unsigned)getUInt(); }
template <>
inline unsigned long long Json::get<unsigned long long>() const { return getUInt(); }
template <>
inline Json Json::get<Json>() const { return *this; }
template <>
inline std::vector<float> Json::get<std::vector<float>>() const {
  std::vector<float> v;
  for (double x : getDoubleVector()) v.push_back((float)x);
  return v;
}
template <>
inline std::vector<int> Json::get<std::vector<int>>() const {
  std::vector<int> v;
  for (const Json &x : elements()) v.push_back((int)x.getInt());
  if (!is_array()) throw std::runtime_error("JSON value is not an array");
  return v;
}
template <>
inline std::vector<size_t> Json::get<std::vector<size_t>>() const {
  std::vector<size_t> v;
  for (const Json &x : elements()) v.push_back((size_t)x.getUInt());
  if (!is_array()) throw std::runtime_error("JSON value is not an array");
  return v;
}
template <>
inline std::vector<std::string> Json::get<std::vector<std::string>>() const {
  std::vector<std::string> v;
  for (const Json &x : elements()) v.push_back(x.getString());
  if (!is_array()) throw std::runtime_error("JSON value is not an array");
  return v;
}
template <>
inline std::vector<std::vector<double>> Json::get<std::vector<std::vector<double>>>() const {
  std::vector<std::vector<double>> v;
  for (const Json &x : elements()) v.push_back(x.getDoubleVector());
  if (!is_array()) throw std::runtime_error("JSON value is not an array");
  return v;
}
template <>
inline std::vector<std::vector<float>> Json::get<std::vector<std::vector<float>>>() const {
  std::vector<std::vector<float>> v;
  for (const Json &x : elements()) v.push_back(x.get<std::vector<float>>());
  if (!is_array()) throw std::runtime_error("JSON value is not an array");
  return v;
}

}  // namespace korali
