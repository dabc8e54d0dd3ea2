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

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : t_(Type::Bool), b_(b) {}
  Json(int v) : t_(Type::Int), i_(v) {}
  Json(long v) : t_(Type::Int), i_(v) {}
  Json(long long v) : t_(Type::Int), i_(v) {}
  Json(unsigned v) : t_(Type::UInt), u_(v) {}
  Json(unsigned long v) : t_(Type::UInt), u_(v) {}
  Json(unsigned long long v) : t_(Type::UInt), u_(v) {}
  Json(double v) : t_(Type::Double), d_(v) {}
  Json(float v) : t_(Type::Double), d_(v) {}
  Json(const char *s) : t_(Type::String), s_(s) {}
  Json(const std::string &s) : t_(Type::String), s_(s) {}
  Json(void (*fn)(Sample &));  // registers the function, stores its index
  template <typename T>
  Json(const std::vector<T> &v) : t_(Type::Array) {
    for (const auto &x : v) a_.emplace_back(x);
  }

  static Json array() {
    Json j;
    j.t_ = Type::Array;
    return j;
  }
  static Json object() {
    Json j;
    j.t_ = Type::Object;
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
  bool contains(const std::string &key) const { return t_ == Type::Object && o_.count(key) != 0; }
  void erase(const std::string &key) {
    if (t_ == Type::Object) o_.erase(key);
  }
  size_t size() const { return t_ == Type::Array ? a_.size() : t_ == Type::Object ? o_.size() : 0; }
  void push_back(const Json &v) {
    if (t_ == Type::Null) t_ = Type::Array;
    if (t_ != Type::Array) throw std::runtime_error("push_back on a non-array JSON value");
    a_.push_back(v);
  }
  const std::map<std::string, Json> &items() const { return o_; }
  const std::vector<Json> &elements() const { return a_; }

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
  bool operator==(const char *v) const { return is_string() && s_ == v; }
  bool operator==(const std::string &v) const { return is_string() && s_ == v; }
  bool operator==(bool v) const { return is_bool() && b_ == v; }
  bool operator==(double v) const { return is_number() && getDouble() == v; }
  bool operator==(int v) const { return is_number() && getDouble() == (double)v; }
  template <typename T>
  bool operator!=(const T &v) const {
    return !(*this == v);
  }

  std::string dump(int indent = -1) const;

 private:
  Type t_ = Type::Null;
  bool b_ = false;
  long long i_ = 0;
  unsigned long long u_ = 0;
  double d_ = 0.0;
  std::string s_;
  std::vector<Json> a_;
  std::map<std::string, Json> o_;
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
