"""Summarise a rocprofv3 --kernel-trace CSV per kernel (count, avg, median, min, max µs)."""
import csv
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("tsa::(anonymous namespace)::", "")
    return name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]


def main(path, title="", skip_first=0):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(f"### {title or path}\n")
    print("| kernel | calls | avg µs | median µs | min µs | max µs | total ms |")
    print("|---|---|---|---|---|---|---|")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v2 = v[skip_first:] if len(v) > skip_first else v
        print(f"| `{k[:70]}` | {len(v)} | {statistics.mean(v):.2f} | {statistics.median(v):.2f} | "
              f"{min(v):.2f} | {max(v):.2f} | {sum(v) / 1000:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
