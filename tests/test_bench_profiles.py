"""bench.py quotes rocprof counters (profiles/{traffic,valu}_by_kernel.json) only
for the source they were measured on: each entry carries the kernel's source
hash (translation unit + the csrc headers it includes + planner + launch code +
build.sh), and an entry whose hash differs from the loaded kernel's reads as
null with the reason "stale" (VERDICT r05 item 2)."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_matching_hash_is_quoted_and_mismatch_is_stale(monkeypatch):
    h = bench.kernel_src_hash("dual_fill_ck_kernel<1>")
    assert h and len(h) == 16
    entry = {"value": 123, "profile": "rX_cfg2", "src_hash": h}
    monkeypatch.setattr(bench, "load_profile", lambda name, tag: dict(entry))
    e, why = bench.profile_entry("traffic_by_kernel.json", "dual_fill_ck_kernel<1>", "t")
    assert e["value"] == 123 and why is None
    entry["src_hash"] = "0" * 16
    e, why = bench.profile_entry("traffic_by_kernel.json", "dual_fill_ck_kernel<1>", "t")
    assert e is None and why.startswith("stale")
    del entry["src_hash"]  # entries from before the hashes: stale too
    e, why = bench.profile_entry("valu_by_kernel.json", "dual_fill_ck_kernel<1>", "t")
    assert e is None and why.startswith("stale")
    monkeypatch.setattr(bench, "load_profile", lambda name, tag: None)
    e, why = bench.profile_entry("valu_by_kernel.json", "dual_fill_ck_kernel<1>", "t")
    assert e is None and why.startswith("not profiled")


def test_hash_follows_included_headers(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(bench.CSRC, csrc)
    build = tmp_path / "build.sh"
    shutil.copy(os.path.join(ROOT, "build.sh"), build)
    h0 = bench.kernel_src_hash("traceback_ck_kernel", str(csrc), str(build))
    assert h0 == bench.kernel_src_hash("traceback_ck_kernel")
    with open(csrc / "ta_layout.h", "a") as f:  # included by ta_walk_ck.hip through ta_device.h
        f.write("\n// edit\n")
    h1 = bench.kernel_src_hash("traceback_ck_kernel", str(csrc), str(build))
    assert h1 != h0
    # another kernel's translation unit does not move it
    with open(csrc / "ta_flex.hip", "a") as f:
        f.write("\n// edit\n")
    assert bench.kernel_src_hash("traceback_ck_kernel", str(csrc), str(build)) == h1
    with open(build, "a") as f:  # nor do build flags leave it unchanged
        f.write("\n# edit\n")
    assert bench.kernel_src_hash("traceback_ck_kernel", str(csrc), str(build)) != h1
