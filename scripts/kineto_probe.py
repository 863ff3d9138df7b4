"""Probe: does torch.profiler (kineto / rocprofiler on ROCm) see the kernels of replayed HIP graphs,
with device timestamps, stream ids and grid sizes?  Prints a short summary."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tspm_amd  # noqa: E402
from oracle import avmnist_ref as orc  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
opt = tspm_amd.FusedAdam(m.parameters(), lr=5e-4, weight_decay=1e-4)
st = tspm_amd.FusedTrainStep(m, opt, None, 128)
a, i, l, _ = orc.synthetic_batch(128, seed=1)
st.load_batch(a.to(dev), i.to(dev), l.to(dev))
for _ in range(5):
    st.run()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
t0 = time.time()
with profile(activities=[ProfilerActivity.CUDA]) as prof:
    for _ in range(3):
        st.run()
    torch.cuda.synchronize()
print("profile wall", time.time() - t0)
evs = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
print("device events", len(evs))
names = {}
for e in evs:
    names.setdefault(e.name, []).append(e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total)
for n, v in sorted(names.items(), key=lambda kv: -sum(kv[1]))[:15]:
    print(f"{len(v):5d} {sum(v)/3:10.1f} us/step  {n[:90]}")
path = "gpurun_out/kineto_probe_trace.json"
os.makedirs("gpurun_out", exist_ok=True)
prof.export_chrome_trace(path)
with open(path) as f:
    tr = json.load(f)
ks = [e for e in tr["traceEvents"] if e.get("cat") == "kernel"]
print("trace kernels", len(ks))
if ks:
    print(json.dumps(ks[0])[:800])
    streams = {}
    for e in ks:
        s = e.get("args", {}).get("stream")
        streams[s] = streams.get(s, 0) + 1
    print("streams", streams)
os.remove(path)
