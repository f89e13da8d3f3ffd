"""Per-update device time of kernel groups from kt_sum.sh runs: python scripts/ks_summary.py DIR..."""
import glob, json, re, sqlite3, sys

GROUPS = {"fy_final+adv": r"k_fy_final|k_adv_epoch\(", "fy_all": r"k_fy|k_scan|k_adv_epoch", "expand_J": r"k_expand_J",
          "minibatch": r"k_minibatch", "rollout": r"rollout_mfma", "all": r"."}
for d in sys.argv[1:]:
    db = sqlite3.connect(glob.glob(d + "/**/*.db", recursive=True)[0])
    rows = db.execute("select name, duration from kernels").fetchall()
    nupd = sum(1 for n, _ in rows if "rollout" in n)
    out = {k: round(sum(du for n, du in rows if re.search(rx, n)) / 1e3 / nupd, 1) for k, rx in GROUPS.items()}
    ms = None
    for line in open(d + ".log"):
        if line.startswith("{"):
            ms = json.loads(line)["ms_per_step"]
    print(d, "us/update", out, "ms_per_step(traced)", ms)
