"""The range proofs behind the packed local fills' three-input max on f16 bit
patterns (ta_layout.h local_max3_offset, ta_planner.cpp flex_local_fits),
checked by brute force on CPU: every biased value and candidate of the local
DP (rows up to n + 15, '-' in targets, random scores including mismatch above
match and positive gaps) lies in [0, 0x7BFF] whenever the bound admits the
shape (tests/cpp/range_proofs.cpp)."""
import os
import subprocess

from conftest import ROOT

CS = os.path.join(ROOT, "bioinfo1_amd", "csrc")


def test_range_proofs(tmp_path):
    exe = str(tmp_path / "range_proofs")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", CS, os.path.join(ROOT, "tests", "cpp", "range_proofs.cpp"),
                           os.path.join(CS, "ta_planner.cpp"), "-o", exe])
    r = subprocess.run([exe, "2000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
