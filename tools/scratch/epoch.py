import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch, torch.nn.functional as F
from ppnp_amd import train as T
from ppnp_amd.model import APPNP, PPNP
adj, attr, labels = T.load_dataset("cora_ml")
dev = torch.device("cuda")
X = torch.FloatTensor(np.asarray(T.normalize_attributes(attr).todense())).to(dev)
y = torch.LongTensor(labels).to(dev)
idx = torch.arange(140, device=dev); idx2 = torch.arange(500, device=dev)
def run(model, n=300, evals=2):
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    for it in range(2):
        torch.cuda.synchronize(); t = time.perf_counter()
        for e in range(n):
            model.train(); lg = model(X, idx); loss = F.cross_entropy(lg, y[idx]) + 0.0025 * model.get_norm()
            opt.zero_grad(); loss.backward(); opt.step(); a = float((lg.argmax(-1) == y[idx]).float().mean())
            model.eval()
            with torch.no_grad():
                for _ in range(evals):
                    l2 = model(X, idx2); float(F.cross_entropy(l2, y[idx2]))
        torch.cuda.synchronize(); dt = (time.perf_counter() - t) / n
    return dt * 1e3
ppr = T._dense_ppr(adj, 0.1)
print("ppnp  ms/epoch %.3f" % run(PPNP(X.shape[1], 7, ppr).to(dev)))
print("appnp ms/epoch %.3f" % run(APPNP(X.shape[1], 7, adj).to(dev)))
print("appnp 0 evals  %.3f" % run(APPNP(X.shape[1], 7, adj).to(dev), evals=0))
m = APPNP(X.shape[1], 7, adj).to(dev); H = torch.randn(2810, 7, device=dev)
from ppnp_amd.ops import propagate_forward
for _ in range(10): propagate_forward(m.graph(), H, 10, 0.1)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(300): propagate_forward(m.graph(), H, 10, 0.1)
torch.cuda.synchronize(); print("propagate_forward call ms %.3f" % ((time.perf_counter() - t) / 300 * 1e3))
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    run(APPNP(X.shape[1], 7, adj).to(dev), n=50)
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
