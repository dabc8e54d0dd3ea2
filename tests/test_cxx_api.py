"""The C++ user API in the reference's own idioms (SURVEY.md §8 b): a problem
definition written like examples/features/running.cxx (float x =
k["Parameters"][0]; &direct as the objective; auto e = korali::Experiment();
variadic KORALI_GET; Sample::update; Experiment::getEvaluation) compiled
against korali.hpp and linked with libkorali_engine.so, plus the Python
surface of the same checks."""
import os
import subprocess

import pytest

from korali_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def example():
    exe = _build.CXX_EXAMPLE
    if not os.path.exists(exe):
        _build.build_cxx_example()
    return exe


def test_reference_idioms_compile_and_cpu_checks(tmp_path):
    r = subprocess.run([example(), "cpu"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "REFERENCE_IDIOMS PASS" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_reference_idioms_run_cmaes_direct(tmp_path):
    r = subprocess.run([example(), "gpu"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "REFERENCE_IDIOMS PASS (cpu+gpu)" in r.stdout, r.stdout + r.stderr


def _experiment(korali):
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Function"] = lambda s: None
    e["Variables"][0]["Name"] = "X"
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 8
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    return e


def test_python_misspelt_keys_rejected():
    import korali
    k = korali.Engine()
    e = _experiment(korali)
    e["Solver"]["Mu Tipe"] = "Linear"
    with pytest.raises(RuntimeError, match="Unrecognized settings for Korali module: CMAES"):
        k.run(e)
    e = _experiment(korali)
    e["Problem"]["Objective Functon"] = lambda s: None
    with pytest.raises(RuntimeError, match="Unrecognized settings for Korali module: Optimization"):
        k.run(e)
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Custom"
    e["Problem"]["Likelihood Model"] = lambda s: None
    e["Distributions"][0]["Name"] = "U"
    e["Distributions"][0]["Type"] = "Univariate/Uniform"
    e["Distributions"][0]["Minimum"] = -1.0
    e["Distributions"][0]["Maximum"] = 1.0
    e["Variables"][0]["Name"] = "X"
    e["Variables"][0]["Prior Distribution"] = "U"
    e["Solver"]["Type"] = "Sampler/TMCMC"
    e["Solver"]["Population Size"] = 16
    e["Solver"]["Target Coefficient of Variaton"] = 1.0
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    with pytest.raises(RuntimeError, match="Unrecognized settings for Korali module: TMCMC"):
        k.run(e)


def test_python_get_evaluation_and_sample_update():
    import korali
    e = _experiment(korali)
    with pytest.raises(RuntimeError, match="This solver does not support evaluation operations."):
        e.getEvaluation([[[1.0]]])
    s = korali.Sample()
    s["Parameters"] = [1.0]
    s.update()
    assert s["Parameters"][0] == 1.0
