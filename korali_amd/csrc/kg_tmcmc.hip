// kg_tmcmc.hip — TMCMC generation (TMCMC.cpp.base:107-381) on the device.
// (placeholder entry points; the device TMCMC path lands in the next step)
#include "../../include/korali_amd.h"
#include "kg_common.hpp"

struct kg_tmcmc_s {
  int dummy;
};

extern "C" {
#define KG_TMCMC_TODO \
  kg::set_error("kg_tmcmc: device TMCMC path not built yet"); \
  return 1;
int kg_tmcmc_create(const kg_tmcmc_cfg *, kg_tmcmc_t *) { KG_TMCMC_TODO }
int kg_tmcmc_destroy(kg_tmcmc_t) { return 0; }
int kg_tmcmc_generation(kg_tmcmc_t, size_t) { KG_TMCMC_TODO }
int kg_tmcmc_synchronize(kg_tmcmc_t) { KG_TMCMC_TODO }
int kg_tmcmc_field_size(kg_tmcmc_t, const char *, size_t *) { KG_TMCMC_TODO }
int kg_tmcmc_get_field(kg_tmcmc_t, const char *, double *, size_t) { KG_TMCMC_TODO }
int kg_tmcmc_set_field(kg_tmcmc_t, const char *, const double *, size_t) { KG_TMCMC_TODO }
int kg_tmcmc_get_rng(kg_tmcmc_t, int, void *) { KG_TMCMC_TODO }
int kg_tmcmc_set_rng(kg_tmcmc_t, int, const void *) { KG_TMCMC_TODO }
int kg_tmcmc_prepare(kg_tmcmc_t, size_t) { KG_TMCMC_TODO }
int kg_tmcmc_evaluate(kg_tmcmc_t) { KG_TMCMC_TODO }
int kg_tmcmc_process(kg_tmcmc_t, size_t) { KG_TMCMC_TODO }
}
