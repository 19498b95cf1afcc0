"""Host-side pieces of bench.py (no GPU): the PMC summary lookup that fills the
bench line's `roofline.traffic` / `mfma_busy`."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pmc_lookup_exact_and_defaulted_template_args():
    table = {
        "k_conv_x3<9,3,18,1,2,2,false,true,false>": 1,
        "k_conv_x3<9,3,18,1,2,2,false,false,false>": 2,
        "k_conv_x3<9,3,18,1,2,2,false,false,true>": 3,
        "k_sp50_dx<3>": 4,
    }
    assert bench.pmc_lookup(table, "k_sp50_dx<3>") == 4
    # the timing names omit trailing template arguments left at false
    assert bench.pmc_lookup(table, "k_conv_x3<9,3,18,1,2,2,false,true>") == 1
    assert bench.pmc_lookup(table, "k_conv_x3<9,3,18,1,2,2,false,false>") == 2
    # a non-default trailing argument is a different kernel
    assert bench.pmc_lookup({"k_conv_x3<9,3,18,1,2,2,false,false,true>": 3},
                            "k_conv_x3<9,3,18,1,2,2,false,false>") is None
    assert bench.pmc_lookup(table, "k_wgrad_x3<18,1,2,2>") is None
    # round 6: k_conv_x3's trailing wave count (NW = 8 by default, 4 for the
    # two-workgroups-per-CU forward) -- 8 is a default, 4 a different kernel
    t6 = {"k_conv_x3<9,3,18,1,2,2,false,true,false,8>": 5,
          "k_conv_x3<9,3,18,1,2,2,false,false,false,4>": 6}
    assert bench.pmc_lookup(t6, "k_conv_x3<9,3,18,1,2,2,false,true>") == 5
    assert bench.pmc_lookup(t6, "k_conv_x3<9,3,18,1,2,2,false,false>") is None


def test_pmc_profile_needs_this_source_hash(tmp_path, monkeypatch):
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_old_cfg2.json").write_text(json.dumps(
        {"config": "cfg2", "src_sha16": "0" * 16, "hbm_bytes_per_launch": {}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "source_sha16", lambda: "f" * 16)
    data, why = bench.pmc_profile("cfg2")
    assert data is None and "no PMC pass" in why
    (prof / "pmc_new_cfg2.json").write_text(json.dumps(
        {"config": "cfg2", "src_sha16": "f" * 16, "hbm_bytes_per_launch": {"k": 1}}))
    data, src = bench.pmc_profile("cfg2")
    assert data["hbm_bytes_per_launch"] == {"k": 1} and src.endswith("pmc_new_cfg2.json")
