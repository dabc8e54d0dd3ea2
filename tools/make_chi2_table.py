"""The chi-square 0.68 quantiles used by mTMCMC's proposal correction
(gsl_cdf_chisq_Pinv(0.68, N), TMCMC.cpp.base:499) for N = 1..128, printed
as C initialisers (shortest round-trip reprs) for oracle/refcpu.c and
korali_amd/csrc/kg_mtmcmc.hpp.  GSL's own iterative inverse is not
available here: parity with it is unpinned."""
from scipy.stats import chi2

vals = [chi2.ppf(0.68, n) for n in range(1, 129)]
for i in range(0, 128, 4):
    print("  " + ", ".join(repr(float(v)) for v in vals[i:i + 4]) + ",")
