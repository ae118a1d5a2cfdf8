"""CPU: the device restatement of the host libm's expf (hip_llama.cpp_amd/csrc/libm_exact.hpp, used
by the int8 path's softmax and SwiGLU so they compute what runq.c computes) is bit-identical to
this host's expf — on a strided sample of all 2^32 inputs here (tools/probes/expf_exact.cpp runs
the exhaustive check: 0 mismatches) — and its table is the correctly rounded 2^(i/32)."""
import os
import re
import struct
import subprocess
from decimal import Decimal, getcontext

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "hip_llama.cpp_amd", "csrc", "libm_exact.hpp")


def test_table_is_the_correctly_rounded_powers():
    src = open(HDR).read()
    vals = [int(v, 16) for v in re.findall(r"0x([0-9a-f]{16})ull", src)]
    assert len(vals) == 32
    getcontext().prec = 60
    for i, v in enumerate(vals):
        d = float(Decimal(2) ** (Decimal(i) / 32))  # Decimal -> float rounds correctly
        assert struct.unpack("<Q", struct.pack("<d", d))[0] - (i << 47) == v, i


def test_matches_host_expf_on_a_sample(tmp_path):
    exe = tmp_path / "expf_exact"
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-I", os.path.dirname(HDR),
                    os.path.join(REPO, "tools", "probes", "expf_exact.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "1021"], capture_output=True, text=True, timeout=600)  # ~4.2M inputs
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout
