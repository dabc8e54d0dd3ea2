"""One HIP runtime per process (korali_amd/__init__.py): importing korali
before torch must not map a second libamdhip64 / libhsa-runtime64 (two
runtimes disagreed on the occupancy of the multi-workgroup
tridiagonalisation, round 3).  CPU-only: it inspects /proc/self/maps."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import importlib, sys
for m in sys.argv[1:]:
    importlib.import_module(m)
maps = open("/proc/self/maps").read().splitlines()
libs = {l.split()[-1] for l in maps if "libamdhip64" in l or "libhsa-runtime64" in l}
print(len([p for p in libs if "amdhip64" in p]), len([p for p in libs if "hsa-runtime64" in p]))
"""


def mapped(*mods):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("KORALI_AMD_HIP_RUNTIME", None)
    out = subprocess.run([sys.executable, "-c", PROBE, *mods], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return tuple(int(v) for v in out.stdout.split())


def test_korali_then_torch_maps_one_hip_runtime():
    assert mapped("korali", "torch") == (1, 1)


def test_native_then_torch_maps_one_hip_runtime():
    assert mapped("korali_amd.native", "torch") == (1, 1)


PRELOADED = r"""
import ctypes, sys
ctypes.CDLL("/opt/rocm/lib/libhsa-runtime64.so.1", mode=ctypes.RTLD_GLOBAL)  # as rocprofv3's tool does
import korali_amd.native as n
n.lib()
maps = open("/proc/self/maps").read().splitlines()
libs = {l.split()[-1] for l in maps if "libamdhip64" in l or "libhsa-runtime64" in l}
print(sorted(libs))
"""


def test_a_preloaded_system_hsa_keeps_its_hip_runtime():
    """under rocprofv3 the tool maps /opt/rocm's HSA first: the package must
    then bind to /opt/rocm's HIP too, not load torch's on top (two HSA
    runtimes faulted at exit, profiles/r5/c4_teardown_segv.txt)"""
    if not os.path.exists("/opt/rocm/lib/libhsa-runtime64.so.1"):
        return
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("KORALI_AMD_HIP_RUNTIME", None)
    out = subprocess.run([sys.executable, "-c", PRELOADED], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    libs = eval(out.stdout.strip().splitlines()[-1])
    assert len([p for p in libs if "amdhip64" in p]) == 1, libs
    assert len([p for p in libs if "hsa-runtime64" in p]) == 1, libs
    assert not any("torch" in p for p in libs), libs
