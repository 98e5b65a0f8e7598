"""On-disk dataset format and ingestion (hgnn_amd/dataset.py), on the CPU.

* GraphPack round trip: what is written is what is read back, bit for bit, and
  the native CSR batches made from the memory-mapped pack hold exactly the row
  lists of a CsrBatch made from the in-memory graphs; the dense path gives the
  reference's prepare_batch 11-tuple of the same graphs.
* prepare_experiment_sets: the reference's sizes and order
  (preprocessing/loading.py:19-37), shuffled with the same `random` state.
* read_xyz on a QM9-format record (the '*^' exponents included) and the target /
  one-hot / last-atom-only feature semantics of molecule_to_instance
  (preprocessing/preprocessing.py:25-94).  The rdkit-derived part (bond graph and
  atom order from the SMILES) is not restated: parity unpinned, documented.
"""

import random

import numpy as np
import pytest
import torch


def _graphs():
    import hgnn_amd.datagen as dg
    gs = dg.qm9_shape_dataset(9, seed=21)
    gs.append((torch.eye(1, 5), torch.zeros(1, 1), torch.randn(13)))  # single isolated node
    return gs


def test_graphpack_round_trip(tmp_path):
    from hgnn_amd.dataset import GraphPack
    gs = _graphs()
    pack = GraphPack.write(str(tmp_path / "p"), gs)
    assert len(pack) == len(gs)
    for i, (x, a, t) in enumerate(gs):
        x2, a2, t2 = pack.graph(i)
        assert torch.equal(x2, x.float()) and torch.equal(a2, a.float()) and torch.equal(t2, t.float())
    # reopening maps the same files; nothing is unpickled
    again = GraphPack(str(tmp_path / "p"))
    assert again.meta["graphs"] == len(gs) and again.meta["features"] == 5


def test_graphpack_accepts_reference_instances(tmp_path):
    from functions.operators import graph_operators
    from hgnn_amd.dataset import GraphPack
    gs = _graphs()[:4]
    inst = [[x, a, t, *graph_operators([x, a], 1, True)] for x, a, t in gs]
    pack = GraphPack.write(str(tmp_path / "p"), inst)
    rebuilt = pack.instances(range(len(gs)))
    for r, o in zip(rebuilt, inst):
        for u, v in zip(r, o):
            assert torch.equal(u, v)


def test_graphpack_batches_match_in_memory(tmp_path):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    from hgnn_amd.csr import CsrBatch
    from hgnn_amd.dataset import GraphPack
    gs = _graphs()
    pack = GraphPack.write(str(tmp_path / "p"), gs)
    order = [3, 0, 7, 9, 1, 5, 2]
    got = list(pack.batches(order, 4, task=2, device="cpu"))
    assert [b.bs for b in got] == [4, 3]
    for b, part in zip(got, [order[:4], order[4:]]):
        ref = CsrBatch([(gs[i][0], gs[i][1]) for i in part], device="cpu",
                       targets=torch.tensor([float(gs[i][2][2]) for i in part]))
        assert torch.equal(b.image, ref.image) and torch.equal(b.T, ref.T)
    dense = list(pack.batches(order, 4, task=2, dense=True))
    inst = [[gs[i][0], gs[i][1], gs[i][2], *graph_operators([gs[i][0], gs[i][1]], 1, True)] for i in order[:4]]
    ref = prepare_batch(inst, 2, 1)
    for u, v in zip(dense[0], ref):
        assert torch.equal(u, v)


@pytest.mark.parametrize("n", [0, 1, 9, 10, 11, 107])
def test_prepare_experiment_sets(n):
    from hgnn_amd.dataset import prepare_experiment_sets
    data = list(range(n))
    tr, va, te = prepare_experiment_sets(list(data))
    assert (len(tr), len(va), len(te)) == (int(0.8 * n), int(0.1 * n), n - int(0.8 * n) - int(0.1 * n))
    assert tr + va + te == data
    random.seed(4)
    tr, va, te = prepare_experiment_sets(list(data), shuf=True)
    random.seed(4)
    expect = list(data)
    random.shuffle(expect)
    assert tr + va + te == expect


XYZ = """5
gdb 7 1.1705 0.84 0.4 2.7 13.3 -0.2 0.03 0.23 58.5 0.048 -116.4 -116.3 -116.3 -116.4 6.3
C\t-0.0127\t1.0858\t0.008\t-0.535
N\t0.0021\t-0.0043\t0.0021\t-0.2*^-2
H\t1.0117\t1.4638\t0.0003\t0.133
H\t-0.5408\t1.4475\t-0.8766\t0.133
H\t-0.5238\t1.4379\t0.9064\t0.1.*^-1
1341.3\t1341.5\t3271.8
C[NH2]\tC[NH2]
InChI=1S/CH5N/c1-2/h2H2,1H3\tInChI=1S/CH5N/c1-2/h2H2,1H3
"""


def test_read_xyz_and_instance():
    from hgnn_amd.dataset import atom_one_hot, molecule_instance, molecule_targets, read_xyz
    mol = read_xyz(XYZ)
    assert mol["Na"] == 5 and mol["tag"] == "gdb" and mol["ident"] == 7 and mol["smiles"] == "C[NH2]"
    assert mol["atoms"][1][2] == pytest.approx(-0.2e-2)   # '*^' exponent
    assert mol["atoms"][4][2] == pytest.approx(0.1e-1)    # '.*^' exponent
    assert mol["alpha"] == 13.3 and mol["Cv"] == 6.3 and mol["freq"][-1] == 3271.8
    t = molecule_targets(mol)
    np.testing.assert_allclose(t.numpy(), np.float32([13.3, 6.3, -116.4, 0.23, -116.3, -0.2, 0.03, 2.7, 3271.8,
                                                      58.5, -116.3, -116.4, 0.048]))
    assert torch.equal(atom_one_hot(["H", "C", "N", "O", "F"]), torch.eye(5))
    x, a, t2 = molecule_instance(mol, [(0, 1, 1.0), (0, 2, 1.0), (0, 3, 1.0)], spatial=True, charge=True)
    assert x.shape == (5, 9) and torch.equal(t2, t)
    # only the last atom carries coordinates and charge (the reference's indentation)
    assert torch.all(x[:4, 5:] == 0) and x[4, 5] == pytest.approx(-0.5238) and x[4, 8] == pytest.approx(0.01)
    assert a[0, 1] == 1 and a[1, 0] == 1 and a.sum() == 6
