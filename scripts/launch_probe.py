import sys, time, os
sys.path.insert(0, "fft-wavespec_amd")
import torch
from wavespec_amd import bridge, synth
dev = torch.device("cuda", 0)
n, w = 4096, 65536
s = synth.random_walk_torch(n * w, 11, dev)
o = torch.empty(w * n // 2, dtype=torch.float64, device=dev)
plan = bridge.Plan(0, n, n, w, "none", "hann")
st = torch.cuda.current_stream().cuda_stream
for _ in range(5): plan.execute(s.data_ptr(), o.data_ptr(), st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(30): plan.execute(s.data_ptr(), o.data_ptr(), st)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue 30: {(t1-t0)*1e3:.3f} ms ({(t1-t0)/30*1e6:.1f} us each); total {(t2-t0)*1e3:.3f} ms ({(t2-t0)/30*1e3:.4f} ms/step)")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); 
for _ in range(30): plan.execute(s.data_ptr(), o.data_ptr(), st)
e1.record(); e1.synchronize()
print(f"events: {e0.elapsed_time(e1)/30:.4f} ms/step")
# tiny-kernel launch overhead: 1 window
p1 = bridge.Plan(0, n, n, 1, "none", "hann")
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(200): p1.execute(s.data_ptr(), o.data_ptr(), st)
t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
print(f"1-window plan: enqueue {(t1-t0)/200*1e6:.1f} us each, {(t2-t0)/200*1e6:.1f} us per step")
for K in (30, 100, 300):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(K): plan.execute(s.data_ptr(), o.data_ptr(), st)
    torch.cuda.synchronize(); t2 = time.perf_counter()
    e0.record()
    for _ in range(K): plan.execute(s.data_ptr(), o.data_ptr(), st)
    e1.record(); e1.synchronize()
    print(f"K={K}: wall {(t2-t0)/K*1e3:.4f} ms/step, events {e0.elapsed_time(e1)/K:.4f} ms/step")
