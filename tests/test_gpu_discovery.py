"""AMD GPU discovery script (integration/gpu-discovery/amd-gpu-discovery.sh), the
counterpart of the reference's nvidia-gpu-discovery.sh (flink-external-resources/
flink-external-resource-gpu/src/main/resources/nvidia-gpu-discovery.sh): same arguments,
same output.  Runs on the CPU with a stub `amd-smi` on PATH."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "integration", "gpu-discovery", "amd-gpu-discovery.sh")

AMD_SMI_CSV = """gpu,gpu_bdf,gpu_uuid,kfd_id,node_id,partition_id
0,0000:05:00.0,uuid0,1,2,0
1,0000:15:00.0,uuid1,2,3,0
2,0000:65:00.0,uuid2,3,4,0
3,0000:75:00.0,uuid3,4,5,0
"""


@pytest.fixture
def env(tmp_path):
    stub = tmp_path / "bin"
    stub.mkdir()
    (stub / "amd-smi").write_text("#!/bin/bash\ncat <<'X'\n" + AMD_SMI_CSV + "X\n")
    (stub / "amd-smi").chmod(0o755)
    e = dict(os.environ)
    e["PATH"] = f"{stub}:{e['PATH']}"
    return e, tmp_path


def run(env, *args):
    r = subprocess.run(["bash", SCRIPT, *map(str, args)], env=env, capture_output=True, text=True, timeout=30)
    return r.returncode, r.stdout.strip()


def test_non_coordination(env):
    e, _ = env
    assert run(e, 2) == (0, "0,1")
    assert run(e, 4) == (0, "0,1,2,3")
    assert run(e, 0) == (0, "")
    rc, out = run(e, 5)
    assert rc == 1 and out == "Could not get enough GPU resources."
    assert run(e)[0] == 1  # usage


def test_coordination_mode(env):
    e, tmp = env
    f = tmp / "coord"
    assert run(e, 2, "--enable-coordination-mode", "--coordination-file", f) == (0, "0,1")
    assert run(e, 1, "--enable-coordination-mode", "--coordination-file", f) == (0, "2")
    rc, out = run(e, 2, "--enable-coordination-mode", "--coordination-file", f)
    assert rc == 1
    # owners recorded so far: this test process (alive).  A dead owner's index is taken over.
    lines = f.read_text().split("\n")
    dead = subprocess.Popen([sys.executable, "-c", "pass"])
    dead.wait()
    f.write_text("\n".join(l for l in lines if l and not l.startswith("0 ")) + f"\n0 {dead.pid}\n")
    assert run(e, 2, "--enable-coordination-mode", "--coordination-file", f) == (0, "3,0")
