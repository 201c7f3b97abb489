"""HBM traffic per launch from rocprofv3 --pmc CSVs (MI355X_MICROARCH.md §HBM).

  python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
      <kernel-substring> <key> <algorithmic_bytes_per_launch> [out.json]

<kernel-substring> "=k_hier_x" matches that short kernel name exactly (not
k_hier_x2<...>).  <key> is the kernel template the bench launches (bench.py FUSED_KERNEL, e.g.
k_tree_lds_lag<64>); it is stored as "template" with the full Kernel_Name the
counters were taken on and the git sha of the build (env PMC_GIT_SHA: the GPU
box has no .git), so bench.py only reports traffic measured on its kernel.

Counters are collected in SEPARATE passes (FETCH_SIZE uses 3 TCC slots,
WRITE_SIZE 2).  Both are in KiB.  gfx950 correction: FETCH_SIZE reports half
the bytes of a wide coalesced streaming read (16 B/lane) — doubled here;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def short_name(kernel_name):
    """'void tsa::(anonymous namespace)::k_hier_x2<false>(unsigned short*, ...)' -> 'k_hier_x2<false>'"""
    s = kernel_name[5:] if kernel_name.startswith("void ") else kernel_name
    depth, cut = 0, len(s)
    for i, ch in enumerate(s):   # the argument list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and not s[i:].startswith("(anonymous"):
            cut = i
            break
    s = s[:cut]
    return s.replace("tsa::", "").replace("(anonymous namespace)::", "")


def matches(kernel_name, kernel_sub):
    """kernel_sub '=name': the kernel's short name exactly (k_hier_x is not k_hier_x2<...>); else a substring"""
    if kernel_sub.startswith("="):
        return short_name(kernel_name) == kernel_sub[1:]
    return kernel_sub in kernel_name


def per_dispatch(path, counter, kernel_sub, names=None):
    vals = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if not matches(r.get("Kernel_Name", ""), kernel_sub):
            continue
        if r.get("Counter_Name") != counter:
            continue
        if names is not None:
            names.add(r["Kernel_Name"])
        vals[r.get("Dispatch_Id") or r.get("Correlation_Id")] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch_csv, write_csv, kernel_sub, key, alg = sys.argv[1:6]
    out_path = sys.argv[6] if len(sys.argv) > 6 else None
    alg = int(alg)
    names = set()
    f = per_dispatch(fetch_csv, "FETCH_SIZE", kernel_sub, names)
    w = per_dispatch(write_csv, "WRITE_SIZE", kernel_sub, names)
    fetch_b = 2 * 1024 * statistics.median(f)  # gfx950: FETCH_SIZE reads half of wide streaming loads
    write_b = 1024 * statistics.median(w)
    import os
    res = {"kernel": kernel_sub, "template": key, "kernel_names": sorted(names),
           "git_sha": os.environ.get("PMC_GIT_SHA", "unknown"), "dispatches": [len(f), len(w)], "fetch_size_kib_median": statistics.median(f),
           "write_size_kib_median": statistics.median(w), "read_bytes_corrected": fetch_b, "write_bytes": write_b,
           "hbm_bytes_per_launch": int(fetch_b + write_b), "algorithmic_bytes_per_launch": alg,
           "ratio_to_algorithmic": round((fetch_b + write_b) / alg, 4)}
    print(json.dumps(res, indent=1))
    if out_path:
        try:
            d = json.load(open(out_path))
        except Exception:
            d = {"note": "HBM bytes per launch, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, "
                         "FETCH_SIZE x2 (gfx950 wide-load correction), KiB x1024", "kernels": {}}
        d["kernels"][key] = res
        json.dump(d, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
