"""The committed profiles cover the build in the tree: bench.py's default line (config 5, JIT,
plain variant, short circuit, one GPU) looks up its algorithmic work (profiles/alg_work.json),
its PMC profile (profiles/pmc_summary.json) and the code-independent minimum
(profiles/min_work.json) by the build id of the sources it runs (native.codegen_id); a source
edit that changes the emitted code without new profiles would leave the line's roofline fields
null.  Host only."""
import json
import os

from mythril_amd import native, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _entries(name):
    with open(os.path.join(ROOT, "profiles", name)) as f:
        return json.load(f)["entries"]


def test_profiles_cover_the_current_build():
    build = native.codegen_id("jit")
    spec = synth.load_spec()
    alg = [e for e in _entries("alg_work.json")
           if e["codegen_id"] == build and e["variant"] == "plain"]
    assert alg, "profiles/alg_work.json has no entry for build %s: run scripts/alg_work.py" % build
    assert 0 < alg[-1]["alg_lane_ops_per_eval"] <= alg[-1]["exec_lane_ops_per_eval_sc"]
    pmc = [e for e in _entries("pmc_summary.json")
           if e.get("codegen_id") == build and e.get("variant", "plain") == "plain"
           and e.get("engine") == "jit" and e.get("short_circuit")
           and e.get("tapes") == spec["n_tapes"] and e.get("rows_per_gpu") == 1 << 26]
    assert pmc, ("profiles/pmc_summary.json has no PMC profile of build %s: run scripts/"
                 "profile.sh and scripts/summarize_profile.py" % build)
    assert pmc[-1]["hbm_bytes_per_launch"] > 0 and pmc[-1]["exec_lane_ops_per_launch"] > 0
    mw = [e for e in _entries("min_work.json") if e.get("variant") == "plain"]
    assert mw and mw[-1]["min_lane_ops_per_eval"] < alg[-1]["alg_lane_ops_per_eval"]
