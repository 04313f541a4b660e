"""bench._pmc_traffic: a PMC entry (profiles/pmc_traffic.json) counts only for the library build it
was measured on. A stale stamp, a missing stamp or a missing entry gives traffic None and says why,
so counters from other kernels are never carried into the line; the build's own stamp gives the
recorded bytes. Also the population's momentum dtype guard."""
import argparse
import json
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _args(tmp_path, entries):
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(entries))
    return argparse.Namespace(traffic_json=str(p))


def test_stamp_matching_build_carries_traffic(tmp_path):
    import bench
    from evolutionarydistributedtraining_amd._lib import library_sha256
    here = library_sha256()
    assert here is not None, "build() first: the library is the stamp"
    args = _args(tmp_path, {"k": {"hbm_bytes_per_launch": 123.0, "lib_sha256": here}})
    value, note = bench._pmc_traffic(args, "k", with_note=True)
    assert value == 123.0 and here[:12] in note


@pytest.mark.parametrize("stamp", ["0" * 64, None])
def test_stale_or_unstamped_entry_gives_null_traffic(tmp_path, stamp):
    import bench
    entry = {"hbm_bytes_per_launch": 123.0}
    if stamp:
        entry["lib_sha256"] = stamp
    args = _args(tmp_path, {"k": entry})
    value, note = bench._pmc_traffic(args, "k", with_note=True)
    assert value is None and note.startswith("stale")
    assert bench._pmc_traffic(args, "k") is None


def test_missing_entry_or_file_gives_null_traffic(tmp_path):
    import bench
    args = _args(tmp_path, {"other": {"hbm_bytes_per_launch": 1.0}})
    assert bench._pmc_traffic(args, "k", with_note=True) == (None, "no PMC entry for k")
    args = argparse.Namespace(traffic_json=str(tmp_path / "absent.json"))
    value, note = bench._pmc_traffic(args, "k", with_note=True)
    assert value is None and note.startswith("no PMC summary")


def test_committed_summary_entries_are_stamped():
    """Every entry of the committed summary names the build it was measured on."""
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        d = json.load(f)
    for key, entry in d.items():
        if isinstance(entry, dict) and "hbm_bytes_per_launch" in entry:
            assert len(entry.get("lib_sha256") or "") == 64, key


def test_population_rejects_a_separate_momentum_dtype():
    from evolutionarydistributedtraining_amd._lib import EdtError
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    genomes = [{"dna": [i]} for i in range(2)]
    with pytest.raises(EdtError, match="momentum_dtype"):
        ResidentPopulation(ParamLayout([(8,)]), torch.bfloat16, "cpu", genomes, momentum_dtype=torch.float32)
    ResidentPopulation(ParamLayout([(8,)]), torch.bfloat16, "cpu", genomes, momentum_dtype=torch.bfloat16)


def test_population_pmc_attribution_follows_dispatch_order(tmp_path):
    """scripts/pmc_population.py: launches count toward the call they belong to, by dispatch order —
    a call opens at the first pass after a blend (its components' passes follow each other); the
    emitting needed-sums pass (slerp_need_kernel<.., true, ..>) or the co-located pass opens a
    speculative call, a non-emitting needed-sums / triangle Gram pass a two-pass call; the
    member-major blend (both forms) closes it. Other kernels are not counted."""
    import csv
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc_population as P
    launches = [  # (kernel, FETCH_SIZE)
        ("void (anonymous namespace)::slerp_need_kernel<1, 5, true, 1>(Members, NeedSpec)", 100.0),
        ("void (anonymous namespace)::slerp_need_kernel<1, 2, true, 1>(Members, NeedSpec)", 20.0),
        ("(anonymous namespace)::slerp_gram_coef_kernel(double const*)", 1.0),
        ("void (anonymous namespace)::slerp_blend_mm_kernel<1, 1, 5>(Members, PopBlend)", 0.5),
        ("void (anonymous namespace)::slerp_blend_mm_kernel<1, 1, 2>(Members, PopBlend)", 0.25),
        ("void (anonymous namespace)::slerp_pop_stats_lerp_kernel<1, 1>(BlendChildren)", 10.0),
        ("void (anonymous namespace)::slerp_blend_population_kernel<1, 1>(BlendChildren)", 2.0),
        ("void (anonymous namespace)::slerp_need_kernel<1, 8, false, 1>(Members, NeedSpec)", 50.0),
        ("void (anonymous namespace)::slerp_blend_mm_kernel<1, 1, 8>(Members, PopBlend)", 70.0),
        ("void (anonymous namespace)::slerp_gram_kernel<1, 8>(Members)", 5.0),
        ("void at::native::copy_kernel(float)", 1000.0),
    ]
    d = tmp_path / "FETCH_SIZE" / "run"
    d.mkdir(parents=True)
    with open(d / "pmc_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (name, v) in enumerate(launches):
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": name, "Counter_Name": "FETCH_SIZE", "Counter_Value": v})
    got = P.calls(str(tmp_path), "FETCH_SIZE")
    assert got == [["speculative", 100.0 + 20.0 + 0.5 + 0.25], ["speculative", 10.0 + 2.0],
                   ["two_pass", 50.0 + 70.0], ["two_pass", 5.0]]

