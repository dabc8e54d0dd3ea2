// likelihood.cpp — the Bayesian/Reference likelihood models: the user's
// computational model fills a sample's "Reference Evaluations" (and the
// model's dispersion entries), the engine turns them into "logLikelihood"
// against the problem's "Reference Data".
//
// Follows source/modules/problem/bayesian/reference/reference.cpp.base:
//   evaluateLoglikelihood dispatch        :25-44
//   compute_normalized_sse                :46-55
//   Normal                                :57-79   (STDEV_EPSILON clamp :13, _log2pi reference.hpp.base:11)
//   Positive Normal                       :81-108
//   StudentT / Positive StudentT          :110-152
//   Poisson / Geometric                   :154-189
//   Negative Binomial                     :191-229
// and restates the GSL 2.6 functions those call (gsl_ran_tdist_pdf,
// gsl_cdf_tdist_P, gsl_cdf_gaussian_P, gsl_ran_poisson_pdf,
// gsl_ran_geometric_pdf, gsl_sf_lngamma).  Normal is bit-exact against the
// reference's TMCMC result files (tests/python/plot/tmcmc); the other
// models follow GSL's published algorithms, checked against scipy to 1e-12
// relative (parity with GSL's own special functions is unpinned).
//
// These run on the host thread that called the computational model: the
// per-sample work is O(reference data), the model itself is user code.
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "korali.hpp"

namespace korali {

namespace {

constexpr double kLog2Pi = 1.83787706640934533908193770912476;  // reference.hpp.base:11
constexpr double kStdevEpsilon = 0.00000000001;                 // reference.cpp.base:13

[[noreturn]] void lfail(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw KoraliError(std::string("[Korali] Error: ") + buf);
}

// gsl_sf_lngamma; lgamma_r, not lgamma: the Concurrent conduit calls this
// from several threads and lgamma writes the global signgam
double lngamma(double x) {
  int sign;
  return ::lgamma_r(x, &sign);
}

// KORALI_GET(std::vector<double>, sample, key) with the reference's message
std::vector<double> vec(Sample &s, const char *key, const std::string &model, size_t nd) {
  if (!s.contains(key)) lfail("This Bayesian (%s) problem requires a '%s' entry in the sample.\n", model.c_str(), key);
  Json &j = s[key];
  std::vector<double> v;
  // KORALI_GET(std::vector<double>, ...) (sample.hpp:174-190): only an array converts
  if (!j.is_array())
    lfail("Missing or incorrect value ['%s'] for the sample.\n + Cause: type must be array, but is %s\n", key,
          j.is_number() ? "number" : "not an array");
  for (const Json &x : j.elements()) v.push_back(x.getDouble());
  if (v.size() != nd)
    lfail("This Bayesian (%s) problem requires a %lu-sized %s array. Provided: %lu.\n", model.c_str(), (unsigned long)nd, key,
          (unsigned long)v.size());
  return v;
}

// gsl_ran_tdist_pdf (randist/tdist.c)
double tdistPdf(double x, double nu) {
  const double lg1 = lngamma(nu / 2);
  const double lg2 = lngamma((nu + 1) / 2);
  return (std::exp(lg2 - lg1) / std::sqrt(M_PI * nu)) * std::pow((1 + x * x / nu), -(nu + 1) / 2);
}

// regularized incomplete beta I_x(a, b) by the modified Lentz continued
// fraction, with the symmetry swap for x > (a+1)/(a+b+2) (specfunc/beta_inc.c)
double betaCf(double a, double b, double x) {
  const double tiny = 1e-300;
  double c = 1.0, d = 1.0 - (a + b) * x / (a + 1.0);
  if (std::fabs(d) < tiny) d = tiny;
  d = 1.0 / d;
  double h = d;
  for (int m = 1; m <= 1000; m++) {
    const double m2 = 2.0 * m;
    double aa = m * (b - m) * x / ((a + m2 - 1.0) * (a + m2));
    d = 1.0 + aa * d;
    if (std::fabs(d) < tiny) d = tiny;
    c = 1.0 + aa / c;
    if (std::fabs(c) < tiny) c = tiny;
    d = 1.0 / d;
    h *= d * c;
    aa = -(a + m) * (a + b + m) * x / ((a + m2) * (a + m2 + 1.0));
    d = 1.0 + aa * d;
    if (std::fabs(d) < tiny) d = tiny;
    c = 1.0 + aa / c;
    if (std::fabs(c) < tiny) c = tiny;
    d = 1.0 / d;
    const double del = d * c;
    h *= del;
    if (std::fabs(del - 1.0) < 1e-16) break;
  }
  return h;
}

double betaInc(double a, double b, double x) {
  if (x <= 0.0) return 0.0;
  if (x >= 1.0) return 1.0;
  const double ln = lngamma(a + b) - lngamma(a) - lngamma(b) + a * std::log(x) + b * std::log1p(-x);
  const double pre = std::exp(ln);
  if (x < (a + 1.0) / (a + b + 2.0)) return pre * betaCf(a, b, x) / a;
  return 1.0 - pre * betaCf(b, a, 1.0 - x) / b;
}

// Student-t lower tail P(T <= x) through the regularised incomplete beta.
// NOT GSL-equal: gsl_cdf_tdist_P (cdf/tdist.c) switches to a Cornish-Fisher
// expansion for nu > 30 and x^2 < 10 nu and uses other beta_inc forms on its
// remaining branches; this returns the exact tail on every branch (parity with
// GSL unpinned; the Positive StudentT likelihood is off the north-star path).
double tdistP(double x, double nu) {
  const double t = nu / (nu + x * x);
  const double tail = 0.5 * betaInc(nu / 2, 0.5, t);  // P(T > |x|)
  return x < 0 ? tail : 1.0 - tail;
}

// gsl_cdf_gaussian_P(x, 1.0)
double gaussianP(double x) { return 0.5 * std::erfc(-x / M_SQRT2); }

// gsl_ran_poisson_pdf (randist/poisson.c), k an unsigned int
double poissonPdf(unsigned int k, double mu) {
  if (mu == 0) return k == 0 ? 1.0 : 0.0;
  const double lf = lngamma((double)k + 1.0);  // gsl_sf_lnfact
  return std::exp(std::log(mu) * k - lf - mu);
}

// gsl_ran_geometric_pdf (randist/geometric.c), k an unsigned int
double geometricPdf(unsigned int k, double p) {
  if (k == 0) return 0;
  if (k == 1) return p;
  return p * std::pow(1 - p, k - 1.0);
}

}  // namespace

double referenceLoglikelihood(const std::string &model, const std::vector<double> &y, Sample &s) {
  const size_t nd = y.size();
  if (model == "Normal") {
    auto f = vec(s, "Reference Evaluations", model, nd);
    auto g = vec(s, "Standard Deviation", model, nd);
    double sse = 0.;
    for (size_t i = 0; i < nd; i++) {
      const double diff = (y[i] - f[i]) / g[i];
      sse += diff * diff;
    }
    double loglike = 0.;
    for (size_t i = 0; i < nd; i++) {
      if (g[i] < 0.0) lfail("Negative (%lf) detected for the Standard Deviation.\n", g[i]);
      if (g[i] < kStdevEpsilon) g[i] = kStdevEpsilon;
      loglike -= std::log(g[i]);
    }
    loglike -= 0.5 * (nd * kLog2Pi + sse);
    return loglike;
  }
  if (model == "Positive Normal") {
    auto f = vec(s, "Reference Evaluations", model, nd);
    auto g = vec(s, "Standard Deviation", model, nd);
    double loglike = 0.;
    for (size_t i = 0; i < nd; i++) {
      const double m = f[i], sd = g[i];
      if (sd <= 0.0) lfail("Negative or zero value (%lf) detected for the Standard Deviation.\n", sd);
      if (m < 0.0) lfail("Negative value (%lf) detected in Reference Evaluation.\n", m);
      if (y[i] < 0.0) lfail("Negative value (%lf) detected in Reference Data.\n", y[i]);
      const double z = (y[i] - m) / sd;
      loglike -= 0.5 * (kLog2Pi + z * z);
      loglike -= std::log(sd);
      loglike -= std::log(1. - gaussianP(-m / sd));
    }
    return loglike;
  }
  if (model == "StudentT" || model == "Positive StudentT") {
    const bool positive = model == "Positive StudentT";
    auto f = vec(s, "Reference Evaluations", model, nd);
    auto nu = vec(s, "Degrees Of Freedom", model, nd);
    double loglike = 0.;
    for (size_t i = 0; i < nd; i++) {
      if (nu[i] <= 0.0) lfail("Negative or zero value (%lf) detected for the Degrees Of Freedom.\n", nu[i]);
      if (positive) {
        if (f[i] < 0.0) lfail("Negative value (%lf) detected in Reference Evaluation.\n", f[i]);
        if (y[i] < 0.0) lfail("Negative value (%lf) detected in Reference Data.\n", y[i]);
      }
      loglike += std::log(tdistPdf(y[i] - f[i], nu[i]));
      if (positive) loglike -= std::log(1.0 - tdistP(-f[i], nu[i]));
    }
    return loglike;
  }
  if (model == "Poisson") {
    auto f = vec(s, "Reference Evaluations", model, nd);
    double loglike = 0.;
    for (size_t i = 0; i < nd; i++) {
      if (f[i] <= 0.0) lfail("Negative value (%lf) detected in Reference Evaluation.\n", f[i]);
      if (y[i] < 0.0) lfail("Negative value (%lf) detected in Reference Data.\n", y[i]);
      loglike += std::log(poissonPdf((unsigned int)y[i], f[i]));
    }
    return loglike;
  }
  if (model == "Geometric") {
    auto f = vec(s, "Reference Evaluations", model, nd);
    double loglike = 0.;
    for (size_t i = 0; i < nd; i++) {
      if (f[i] < 0.0) lfail("Negative value (%lf) detected in Reference Evaluation.\n", f[i]);
      if (y[i] < 0.0) lfail("Negative value (%lf) detected in Reference Data.\n", y[i]);
      loglike += std::log(geometricPdf((unsigned int)(y[i] + 1.0), 1.0 / (1.0 + f[i])));
    }
    return loglike;
  }
  if (model == "Negative Binomial") {
    auto f = vec(s, "Reference Evaluations", model, nd);
    auto r = vec(s, "Dispersion", model, nd);
    double loglike = 0.0;
    for (size_t i = 0; i < nd; i++) {
      const double yi = y[i];
      if (yi < 0) lfail("Negative Binomial Likelihood not defined for negative Reference Data (provided %lf.\n", yi);
      loglike -= lngamma(yi + 1.);
      const double m = f[i];
      if (m <= 0) return -INFINITY;
      const double p = m / (m + r[i]);
      loglike += lngamma(yi + r[i]);
      loglike -= lngamma(r[i]);
      loglike += r[i] * std::log(1 - p);
      loglike += yi * std::log(p);
    }
    return loglike;
  }
  lfail("Bayesian problem (%s) not recognized.\n", model.c_str());
}

// the model's per-datum derivative arrays (KORALI_GET of
// std::vector<std::vector<double>>): nd rows of nth values
static std::vector<std::vector<double>> mat(Sample &s, const char *key, size_t nd, size_t nth, const char *what) {
  if (!s.contains(key) || !s[key].is_array())
    lfail("Missing or incorrect value ['%s'] for the sample.\n", key);
  std::vector<std::vector<double>> m;
  for (const Json &row : s[key].elements()) {
    std::vector<double> r;
    if (row.is_array())
      for (const Json &x : row.elements()) r.push_back(x.getDouble());
    m.push_back(r);
  }
  if (m.size() != nd)
    lfail("Bayesian problem requires a gradient of the %s for each reference evaluation (provided %zu required %zu).",
          what, m.size(), nd);
  for (auto &r : m)
    if (r.size() != nth)
      lfail("Bayesian Reference %s gradient calculation requires gradients of size %zu (provided size %zu)\n", what, nth,
            r.size());
  return m;
}

// Reference::evaluateLoglikelihoodGradient, Normal (reference.cpp.base:231-286):
// sum over data of -g'/g + (y - f) f'/g^2 + (y - f)^2 g'/g^3
std::vector<double> referenceLoglikelihoodGradient(const std::string &model, const std::vector<double> &y, Sample &s,
                                                   size_t nth) {
  if (model != "Normal") lfail("Gradient not yet implemented for logLikelihood model of type '%s'.", model.c_str());
  const size_t nd = y.size();
  auto f = vec(s, "Reference Evaluations", model, nd);
  auto g = vec(s, "Standard Deviation", model, nd);
  auto gF = mat(s, "Gradient Mean", nd, nth, "Mean");
  auto gG = mat(s, "Gradient Standard Deviation", nd, nth, "Standard Deviation");
  std::vector<double> out(nth, 0.0);
  for (size_t i = 0; i < nd; ++i) {
    const double inv = 1.0 / g[i], inv2 = inv * inv, inv3 = inv2 * inv;
    const double dif = y[i] - f[i];
    for (size_t d = 0; d < nth; ++d)
      out[d] += -inv * gG[i][d] + inv2 * dif * gF[i][d] + inv3 * dif * dif * gG[i][d];
  }
  return out;
}

// Reference::evaluateFisherInformation, Normal (reference.cpp.base:514-566)
std::vector<double> referenceFisherInformation(const std::string &model, const std::vector<double> &y, Sample &s,
                                               size_t nth) {
  if (model != "Normal") lfail("Fisher Information not yet implemented for logLikelihood model of type '%s'.", model.c_str());
  const size_t nd = y.size();
  auto g = vec(s, "Standard Deviation", model, nd);
  auto gF = mat(s, "Gradient Mean", nd, nth, "Mean");
  auto gG = mat(s, "Gradient Standard Deviation", nd, nth, "Standard Deviation");
  std::vector<double> F(nth * nth, 0.0);
  for (size_t i = 0; i < nd; ++i) {
    const double var = g[i] * g[i], vinv = 1. / var;
    for (size_t k = 0; k < nth; ++k) {
      for (size_t l = 0; l < k; ++l) {
        const double t = vinv * gF[i][k] * gF[i][l] + 2. * vinv * gG[i][k] * gG[i][l];
        F[k * nth + l] += t;
        F[l * nth + k] += t;
      }
      F[k * nth + k] += (vinv * gF[i][k] * gF[i][k] + 2. * vinv * gG[i][k] * gG[i][k]);
    }
  }
  return F;
}

bool isReferenceLikelihoodModel(const std::string &model) {
  for (const char *m : {"Normal", "Positive Normal", "StudentT", "Positive StudentT", "Poisson", "Geometric", "Negative Binomial"})
    if (model == m) return true;
  return false;
}

}  // namespace korali
