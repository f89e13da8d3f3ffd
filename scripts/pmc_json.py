"""Summarise rocprofv3 --pmc CSV passes into pmc_<tag>.json (+ a text
table on stdout) that bench.py reads for the roofline `traffic` fields.

    python scripts/pmc_json.py TAG DIR [DIR ...] > gpurun_out/<tag>_pmc.txt
    (writes gpurun_out/pmc_<tag>.json; copy both under profiles/)

Each DIR holds one pass's *counter_collection.csv.  Per kernel: launches and
the mean of every counter per dispatch (and of the dispatch duration).  HBM bytes per launch:
  FETCH_SIZE (KiB) x 1024 x fetch_correction + WRITE_SIZE (KiB) x 1024,
with fetch_correction = 2 for kernels whose reads are 16-B-per-lane
streaming loads (MI355X_MICROARCH.md HBM: "On gfx950 FETCH_SIZE reports
exactly 1/2 of the bytes of a wide coalesced streaming read ... double it")
and 1 otherwise (64-B row gathers: uncalibrated by the guide; their raw
FETCH matches the 64-B records gathered, so no factor is applied).
MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES (MFMA issue-busy cycles summed over
all SIMDs) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the fraction of SIMD
cycles of the dispatch the matrix cores were busy (GRBM_GUI_ACTIVE is the sum
over the 8 XCDs, MI355X_MICROARCH.md DVFS note); the clock the dispatch ran at
is GRBM_GUI_ACTIVE / 8 / duration.
Each kernel entry records the sha256 of the source file the kernel lives in,
so bench.py can tell a profile of the current code from a stale one.
"""
import csv
import glob
import hashlib
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "burn-ppo_amd", "csrc")
# kernel -> (source file, FETCH correction)
KERNELS = {
    "k_gae_1p_seg": ("k_gae.hip", 2.0),
    "k_gae_1p": ("k_gae.hip", 1.0),
    "k_minibatch_mfma": ("k_update.hip", 1.0),
    "k_minibatch_split": ("k_update.hip", 1.0),
    "k_minibatch_split_exactfwd": ("k_update.hip", 1.0),   # k_minibatch_split<true> (first minibatch)
    "k_cartpole_rollout_mfma": ("k_rollout.hip", 1.0),
    "k_pack_rows": ("k_update.hip", 1.0),
}


def src_sha(fname):
    with open(os.path.join(CSRC, fname), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def short_name(full):
    n = full.split("(")[0]
    n = n.split("::")[-1]
    if n.startswith("k_minibatch_split<true>"):      # the update's first minibatch (exact forward)
        return "k_minibatch_split_exactfwd"
    return n.split("<")[0]


def main():
    tag, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    k = short_name(row["Kernel_Name"])
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    vals[k]["dur_ns"].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    try:
        rev = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                             text=True).stdout.strip()
    except OSError:
        rev = None
    out = {"tag": tag, "git_rev": rev, "kernels": {}}
    print(f"# rocprofv3 --pmc passes {tag} (git {rev}); per-dispatch means")
    for k, cs in sorted(vals.items()):
        if k not in KERNELS:
            continue
        fname, corr = KERNELS[k]
        e = {"source": fname, "source_sha": src_sha(fname), "launches": max(len(v) for v in cs.values())}
        for c, v in cs.items():
            e[c] = sum(v) / len(v)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["fetch_correction"] = corr
            e["traffic_bytes"] = int(e["FETCH_SIZE"] * 1024 * corr + e["WRITE_SIZE"] * 1024)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in e and e.get("GRBM_GUI_ACTIVE", 0) > 0:
            cyc = e["GRBM_GUI_ACTIVE"] / 8.0
            e["mfma_util"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0)
            e["clock_ghz"] = cyc / e["dur_ns"]
        out["kernels"][k] = e
        print(f"{k}: " + ", ".join(f"{c}={v:.6g}" if isinstance(v, float) else f"{c}={v}" for c, v in e.items()))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
