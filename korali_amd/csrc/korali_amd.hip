// korali_amd.hip — single translation unit for the device library
// (one definition of the __constant__ tables shared by every kernel).
#include "kg_common.hip"
#include "kg_mtjump.hip"
#include "kg_rng.hip"
#include "kg_eigen.hip"
#include "kg_cmaes.hip"
#include "kg_tmcmc.hip"
#include "kg_vracer.hip"
