"""Quick GPU probe: HIP runtime interplay (torch first), a plan run, CLI run."""
import os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
print("torch", torch.__version__, torch.version.hip, "cuda avail", torch.cuda.is_available(), flush=True)
print(torch.cuda.get_device_name(0), flush=True)
import __graft_entry__ as g
g.smoke()
import tenstorrentallreduce_amd as t
for argv in (["0","1","2","-1","1","32","0","0"], ["1","1","8","13","5","32","0","1"]):
    p = t.run_cli("allred_BO_2D", argv, env={"ALLRED_REPORT": "1"})
    print(p.returncode, p.stdout.strip()[-200:], p.stderr.strip()[-400:], flush=True)
print("maps:", [l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "rccl" in l or "allred" in l][:20])
