"""Per-iteration cost of Algorithm 1's test in the panel pairs: the C4 shard for 300 iterations
with tol = 0 (fixed N) and tol = 1e-30 (tests every K = 10, nothing converges), one launch
(GPU box: GPAD_PANEL_NOPHASE=1 python tools/tol_cost.py).  Measured: 11.2 vs 10.8 us, i.e. no cost."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'gpu-dualgradient-mpc_amd'))
import torch, bench, gpad_mpc
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tune_env  # noqa: F401,E402  (legacy GPAD_* env -> gpad_set_option)
dev = torch.device('cuda:0')
n = m = 200; B = 8192
ML, G, L, M, g = bench.make_shard(n, m, B, 0)
f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
dML, dG, dM, dg = f32(ML), f32(G), f32(M), f32(g)
z = torch.zeros(B, n, device=dev); y = torch.zeros(B, m, device=dev)
s = gpad_mpc.GpadSolver(0)
s.setup(dML, dG, float(np.float32(L)), n=n, m=m, batch=B, shared=True, check_every=10)
for tol in (0.0, 1e-30):
    best = 1e9
    for _ in range(4):
        st = s.run(z.zero_(), y.zero_(), dM, dg, 300, tol)
        best = min(best, st['kernel_ms'])
    print(json.dumps({'tol': tol, 'us_per_iter': best * 1e3 / 300, 'iters': st['iterations']}))
