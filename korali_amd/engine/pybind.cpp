// pybind.cpp — the `libkorali` Python module (reference: engine.cpp:201-254,
// source/auxiliar/koraliJson.cpp, source/auxiliar/py2json.hpp): Engine,
// Experiment and Sample with the reference's __getitem__ / __setitem__
// behaviour.  Nested keys go through a path proxy, leaves come back as
// Python values, Python callables become entries of the function table.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <variant>

#include "korali.hpp"

namespace py = pybind11;
using korali::Json;

namespace {

Json toJson(const py::handle &o);
bool jsonRefValue(const py::handle &o, Json &out);  // o is a koraliJson proxy: its value

py::object toPy(const Json &j) {
  switch (j.type()) {
    case Json::Type::Null: return py::none();
    case Json::Type::Bool: return py::bool_(j.getBool());
    case Json::Type::Int: return py::int_(j.getInt());
    case Json::Type::UInt: return py::int_(j.getUInt());
    case Json::Type::Double: return py::float_(j.getDouble());
    case Json::Type::String: return py::str(j.getString());
    case Json::Type::Array: {
      py::list l;
      if (const auto *pd = j.packedDoubles()) {
        for (double d : *pd) l.append(d);
        return std::move(l);
      }
      for (const auto &x : j.elements()) l.append(toPy(x));
      return std::move(l);
    }
    case Json::Type::Object: {
      py::dict d;
      for (const auto &kv : j.items()) d[py::str(kv.first)] = toPy(kv.second);
      return std::move(d);
    }
  }
  return py::none();
}

Json toJson(const py::handle &o) {
  if (o.is_none()) return Json();
  {
    Json v;
    if (jsonRefValue(o, v)) return v;
  }
  if (py::isinstance<py::bool_>(o)) return Json(o.cast<bool>());
  if (py::isinstance<py::int_>(o)) {
    const py::int_ i = py::reinterpret_borrow<py::int_>(o);
    if (py::int_(i) < py::int_(0)) return Json((long long)i.cast<long long>());
    return Json((unsigned long long)i.cast<unsigned long long>());
  }
  if (py::isinstance<py::float_>(o)) return Json(o.cast<double>());
  if (py::isinstance<py::str>(o)) return Json(o.cast<std::string>());
  if (py::hasattr(o, "tolist") && !py::isinstance<py::list>(o)) return toJson(o.attr("tolist")());  // numpy
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    Json a = Json::array();
    for (auto x : o) a.push_back(toJson(x));
    return a;
  }
  if (py::isinstance<py::dict>(o)) {
    Json d = Json::object();
    for (auto kv : py::reinterpret_borrow<py::dict>(o)) d[py::str(kv.first).cast<std::string>()] = toJson(kv.second);
    return d;
  }
  if (PyCallable_Check(o.ptr())) {
    py::function f = py::reinterpret_borrow<py::function>(o);
    const size_t idx = korali::registerFunction([f](korali::Sample &s) {
      py::gil_scoped_acquire g;
      f(py::cast(&s, py::return_value_policy::reference));
    });
    return Json((unsigned long long)idx);
  }
  // numpy scalars and other numbers
  if (py::hasattr(o, "__float__")) return Json(o.cast<double>());
  throw std::runtime_error("cannot store a value of type " + std::string(py::str(py::type::handle_of(o))) + " in Korali JSON");
}

using Key = std::variant<std::string, size_t>;

// path proxy into a JSON tree (KoraliJson getItem / setItem)
struct JsonRef {
  Json *root;
  std::vector<Key> path;
  py::object keep;  // keeps the owning Experiment / Sample alive

  Json *find() const {  // nullptr if missing
    const Json *j = root;
    for (const auto &k : path) {
      if (std::holds_alternative<std::string>(k)) {
        if (!j->is_object() || !j->contains(std::get<std::string>(k))) return nullptr;
        j = &j->at(std::get<std::string>(k));
      } else {
        if (!j->is_array() || std::get<size_t>(k) >= j->size()) return nullptr;
        j = &j->at(std::get<size_t>(k));
      }
    }
    return const_cast<Json *>(j);
  }
  Json &make() const {
    Json *j = root;
    for (const auto &k : path) {
      if (std::holds_alternative<std::string>(k))
        j = &(*j)[std::get<std::string>(k)];
      else
        j = &(*j)[std::get<size_t>(k)];
    }
    return *j;
  }
};

bool isContainer(const Json &j) {
  if (j.is_object()) return true;
  if (j.is_array()) return j.size() == 0 || j.elements()[0].is_object();
  return false;
}

py::object child(const JsonRef &r, const Key &k) {
  JsonRef c{r.root, r.path, r.keep};
  c.path.push_back(k);
  Json *j = c.find();
  if (j && !j->is_null() && !isContainer(*j)) return toPy(*j);
  return py::cast(c);
}

Key key(const py::handle &k) {
  if (py::isinstance<py::int_>(k)) {
    const long long i = k.cast<long long>();
    if (i < 0) throw py::index_error("negative index");
    return (size_t)i;
  }
  return k.cast<std::string>();
}

bool jsonRefValue(const py::handle &o, Json &out) {
  if (!py::isinstance<JsonRef>(o)) return false;
  const Json *j = o.cast<const JsonRef &>().find();
  out = j ? *j : Json();
  return true;
}

}  // namespace

PYBIND11_MODULE(libkorali, m) {
  m.doc() = "MI355X-native Korali engine (CMA-ES / TMCMC generation loop on the korali_amd C-ABI)";
  py::register_exception<korali::KoraliError>(m, "KoraliError", PyExc_RuntimeError);

  py::class_<JsonRef>(m, "koraliJson")
      .def("__getitem__", [](const JsonRef &r, py::handle k) { return child(r, key(k)); })
      .def("__setitem__",
           [](const JsonRef &r, py::handle k, py::handle v) {
             JsonRef c{r.root, r.path, r.keep};
             c.path.push_back(key(k));
             c.make() = toJson(v);
           })
      // s["Reference Evaluations"] = []; s["Reference Evaluations"] += [v]
      // (the reference's model scripts): extend the array in place
      .def("__iadd__",
           [](py::object self, py::iterable items) {
             Json &j = self.cast<const JsonRef &>().make();
             if (j.is_null()) j = Json::array();
             if (!j.is_array()) throw py::type_error("+= on a non-array Korali JSON entry");
             for (auto x : items) j.push_back(toJson(x));
             return self;
           })
      .def("__len__", [](const JsonRef &r) { Json *j = r.find(); return j ? j->size() : (size_t)0; })
      .def("__contains__", [](const JsonRef &r, const std::string &k) { Json *j = r.find(); return j && j->contains(k); })
      .def("get", [](const JsonRef &r) { Json *j = r.find(); return j ? toPy(*j) : py::object(py::none()); })
      .def("__repr__", [](const JsonRef &r) { Json *j = r.find(); return j ? j->dump(2) : std::string("null"); });

  py::class_<korali::Sample>(m, "Sample")
      .def(py::init<>())
      .def("__getitem__",
           [](py::object self, py::handle k) {
             auto &s = self.cast<korali::Sample &>();
             return child(JsonRef{&s._js, {}, self}, key(k));
           })
      .def("__setitem__", [](korali::Sample &s, const std::string &k, py::handle v) { s[k] = toJson(v); })
      .def("__contains__", [](korali::Sample &s, const std::string &k) { return s.contains(k); })
      // an environment function's update() waits for the engine: the GIL is
      // released meanwhile (the engine thread never holds it)
      .def("update", [](korali::Sample &s) {
        py::gil_scoped_release nogil;
        s.update();
      });

  py::class_<korali::Experiment>(m, "Experiment")
      .def(py::init<>())
      .def("__getitem__",
           [](py::object self, py::handle k) {
             auto &e = self.cast<korali::Experiment &>();
             return child(JsonRef{&e._js, {}, self}, key(k));
           })
      .def("__setitem__", [](korali::Experiment &e, const std::string &k, py::handle v) { e[k] = toJson(v); })
      .def("loadState", &korali::Experiment::loadState)
      .def("getEvaluation", &korali::Experiment::getEvaluation)
      .def("dump", [](korali::Experiment &e) { return e._js.dump(2); });

  // run() releases the GIL: Python callbacks re-acquire it per sample, so a
  // Concurrent conduit's threads can evaluate samples whose code drops it
  // (NumPy, I/O, native extensions)
  py::class_<korali::Engine>(m, "Engine")
      .def(py::init<>())
      .def("run",
           [](korali::Engine &k, korali::Experiment &e) {
             py::gil_scoped_release nogil;
             k.run(e);
           })
      .def("run",
           [](korali::Engine &k, py::list es) {
             std::vector<korali::Experiment *> v;
             for (auto x : es) v.push_back(&x.cast<korali::Experiment &>());
             py::gil_scoped_release nogil;
             k.run(v);
           })
      .def("__getitem__",
           [](py::object self, py::handle k) {
             auto &e = self.cast<korali::Engine &>();
             return child(JsonRef{&e._js, {}, self}, key(k));
           })
      .def("__setitem__", [](korali::Engine &e, const std::string &k, py::handle v) { e[k] = toJson(v); });

  // test hook: a Bayesian/Reference likelihood model on one sample's entries
  m.def("_reference_loglikelihood", [](const std::string &model, const std::vector<double> &y, py::dict entries) {
    korali::Sample s;
    for (auto kv : entries) s[py::str(kv.first).cast<std::string>()] = toJson(kv.second);
    return korali::referenceLoglikelihood(model, y, s);
  });

  // test hook: Bayesian::evaluate of one parameter vector (CMA-ES on Bayesian problems)
  m.def("_bayesian_evaluate", [](korali::Experiment &e, const std::vector<double> &x) {
    Json out;
    {
      py::gil_scoped_release nogil;  // the model callbacks take the GIL themselves
      out = korali::bayesianEvaluate(e._js, x);
    }
    return toPy(out);
  });

  // test hook: the Distributed conduit's collectives on host data (Host transport)
  m.def("_collective_selftest", [](int port, const std::vector<double> &block, int failRank) {
    korali::CollectiveCheck r;
    {
      py::gil_scoped_release nogil;
      r = korali::collectiveSelfTest(port, block, failRank);
    }
    py::dict d;
    d["rank"] = r.rank;
    d["world"] = r.world;
    d["gathered"] = r.gathered;
    d["summed"] = r.summed;
    d["maxed"] = r.maxed;
    d["peer_failed"] = r.peerFailed;
    return d;
  }, py::arg("port"), py::arg("block"), py::arg("fail_rank") = -1);

  // test hooks: the continuous agent's policy description and initial
  // hyperparameters (pinned against the reference's VRACER result files)
  m.def("_generation_completion_times", [](korali::Experiment &e) { return korali::generationCompletionTimes(e); });
  m.def("_vracer_policy_description", [](korali::Experiment &e) { return toPy(korali::vracerPolicyDescription(e._js)); });
  m.def("_vracer_initial_hyperparameters", [](const std::vector<size_t> &sizes, unsigned seed) {
    return korali::vracerInitialHyperparameters(sizes, seed);
  });

  // test hook: the conduit's batch dispatch with a Python body
  m.def("_conduit_evaluate", [](size_t jobs, size_t n, py::function body) {
    py::gil_scoped_release nogil;
    korali::conduitEvaluate(jobs, n, [&body](size_t i) {
      py::gil_scoped_acquire g;
      body(i);
    });
  });
}
