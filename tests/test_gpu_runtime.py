"""GPU: the deployment's runtime. The JNI shim's libdistml_ps.so runs in a JVM
without torch, on the system ROCm libraries (libamdhip64, librccl from
/opt/rocm) instead of the ones torch bundles. tests/no_torch_worker.py runs the
C-ABI in such a process (a config-2 batch bit-exact against the oracle, and
the native RCCL group at world 1) and reports the libraries it mapped."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_c_abi_without_torch():
    env = dict(os.environ)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "no_torch_worker.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["ok"]
    libs = d["libs"]
    assert "libdistml_ps" in libs and "libamdhip64" in libs, libs
    # not torch's bundled copies (site-packages/torch/lib)
    assert "torch" not in libs["libamdhip64"], libs
    assert "torch" not in libs.get("librccl", ""), libs
    print(json.dumps(libs))
