"""Diagnose HIP-graph capture of executor steps: python tools/graph_diag.py <kind> <mode>
kind: simple | lg ; mode: fwd | step"""
import os
import sys
import faulthandler
faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO, os.path.join(REPO, "tests", "golden")]
import torch  # noqa: E402
import hgnn_amd.datagen as dg  # noqa: E402
from functions.batching import prepare_batch  # noqa: E402
from functions.operators import graph_operators  # noqa: E402
from models.gnns.model_mnb import GNN_lg, GNN_simple  # noqa: E402

kind, mode = sys.argv[1], sys.argv[2]
d = int(sys.argv[3]) if len(sys.argv) > 3 else 2
graphs = dg.sbm_dataset(8, n=30, seed=11) if kind == "simple" else dg.qm9_shape_dataset(64, seed=12)
data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in prepare_batch(data, 0, 1)]
nl = int(sys.argv[4]) if len(sys.argv) > 4 else 6
model = (GNN_simple(0, d, nl, 5, 1, 1) if kind == "simple" else GNN_lg(0, 16, nl, 5, 1, 1, 2)).cuda()
X.requires_grad_(True)
if os.environ.get("DIAG_INIT") == "1":
    import fixture_util as fu
    fu.det_init(model, 13)


def step():
    for p in model.parameters():
        p.grad = None
    X.grad = None
    if mode == "fwd":
        with torch.no_grad():
            model([X, W], Nb, mask) if kind == "simple" else model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        return
    out = model([X, W], Nb, mask) if kind == "simple" else model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    torch.nn.MSELoss()(out, T).backward()
    if os.environ.get("DIAG_KEEP") == "1":
        # DIAG_DETACH=1: keep the values only -- the output's grad_fn keeps the eager step's autograd
        # nodes (the parameters' AccumulateGrad nodes, with the stream they were created on) alive
        buf["out"] = out.detach() if os.environ.get("DIAG_DETACH") == "1" else out


buf = {}
if os.environ.get("DIAG_PRE") == "1":
    step()
    torch.cuda.synchronize()
    print("pre-step ok", flush=True)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print("eager ok", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("replayed ok", kind, mode, d, flush=True)
