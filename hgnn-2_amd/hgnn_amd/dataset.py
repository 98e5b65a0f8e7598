"""On-disk dataset format and ingestion.

The reference keeps datasets as pickled lists of 7-tuples (x, A, t, W, WL, Pm, Pd)
(preprocessing/preprocessing.py:97, functions/data_generator.py:85), splits them
80/10/10 (preprocessing/loading.py:19-37) and builds them from the QM9 `.xyz`
files through rdkit (preprocessing/preprocessing.py:174-275).  Here:

* GraphPack -- a directory of flat `.npy` arrays plus `meta.json`, opened with
  `numpy.load(mmap_mode="r")` (never pickle): packed node features, the
  adjacency as per-graph COO (local i, j, bond order) and the target vectors.
  Only (x, A, t) are stored; the operators W / WL / Pm / Pd are a pure function
  of A and are rebuilt by the native builder when a batch is made, so a pack is
  ~1 % of the pickled 7-tuples (no dense N x N x 3 / M x M x 3 tensors).
* GraphPack.batches -- hgnn_amd.csr.CsrBatch per batch straight from the
  memory-mapped arrays (the executor's layout, csrc/builder.cpp), or the
  reference's dense 11-tuple through functions.batching.prepare_batch.
* prepare_experiment_sets -- the reference split, same sizes and order.
* read_xyz / molecule_targets / atom_one_hot -- the QM9 `.xyz` reader: header
  properties, atoms (with the `*^` exponent form), frequencies and SMILES; the
  13-target vector in molecule_to_instance's order (preprocessing.py:44-57);
  the 5-way atom one-hot (60-77).  The bond graph is NOT derived: the
  reference takes bonds and the atom order from rdkit (AddHs, aromaticity,
  `GetBondTypeAsDouble`, preprocessing.py:238-275), which is absent here, so
  `molecule_instance` takes the bonds as an argument (parity of the rdkit part
  is unpinned).
"""

import json
import os
import random

import numpy as np
import torch

FORMAT = "hgnn-graphpack"
VERSION = 1


def prepare_experiment_sets(data, shuf=False):
    """80/10/10 split of a list, as preprocessing/loading.py:19-37 (in-place random.shuffle when shuf)."""
    n = len(data)
    n_train = int(0.8 * n)
    n_valid = int(0.1 * n)
    if shuf:
        random.shuffle(data)
    return data[:n_train], data[n_train:n_train + n_valid], data[n_train + n_valid:]


class GraphPack:
    """A memory-mapped graph dataset: graphs i = 0 .. len-1 with (x (n_i, f), A (n_i, n_i), t (n_t,))."""

    FILES = ("node_off", "x", "adj_off", "adj_ij", "adj_w", "targets")

    def __init__(self, path):
        with open(os.path.join(path, "meta.json")) as fh:
            meta = json.load(fh)
        if meta.get("format") != FORMAT or meta.get("version") != VERSION:
            raise RuntimeError(f"hgnn_amd: {path} is not a {FORMAT} v{VERSION} directory")
        self.path = path
        self.meta = meta
        arr = {k: np.load(os.path.join(path, k + ".npy"), mmap_mode="r", allow_pickle=False) for k in self.FILES}
        self.node_off = arr["node_off"]
        self.x = arr["x"]
        self.adj_off = arr["adj_off"]
        self.adj_ij = arr["adj_ij"]
        self.adj_w = arr["adj_w"]
        self.targets = arr["targets"]
        g = len(self.node_off) - 1
        if g < 0 or len(self.adj_off) != g + 1 or self.targets.shape[0] != g:
            raise RuntimeError(f"hgnn_amd: inconsistent graph pack {path}")

    @staticmethod
    def write(path, graphs):
        """Write graphs = iterable of (x (n, f), A (n, n), t (n_t,)) -- or the reference's 7-tuples,
        of which only the first three members are kept -- as a pack directory."""
        xs, offs, ij, w, aoff, ts = [], [0], [], [], [0], []
        f = n_t = None
        for inst in graphs:
            x = torch.as_tensor(inst[0]).detach().to("cpu", torch.float32)
            a = torch.as_tensor(inst[1]).detach().to("cpu", torch.float32)
            t = torch.as_tensor(inst[2]).detach().to("cpu", torch.float32).reshape(-1)
            n = x.shape[0]
            if x.dim() != 2 or tuple(a.shape) != (n, n):
                raise RuntimeError(f"hgnn_amd: graph shapes x {tuple(x.shape)}, A {tuple(a.shape)}")
            if f is None:
                f, n_t = x.shape[1], t.numel()
            if x.shape[1] != f or t.numel() != n_t:
                raise RuntimeError("hgnn_amd: every graph needs the same feature and target widths")
            nz = a.nonzero()  # row-major, as A's own order
            xs.append(x.numpy())
            offs.append(offs[-1] + n)
            ij.append(nz.to(torch.int32).numpy().reshape(-1, 2))
            w.append(a[nz[:, 0], nz[:, 1]].numpy())
            aoff.append(aoff[-1] + nz.shape[0])
            ts.append(t.numpy())
        if f is None:
            raise RuntimeError("hgnn_amd: no graphs to write")
        os.makedirs(path, exist_ok=True)
        data = {
            "node_off": np.asarray(offs, dtype=np.int64),
            "x": np.concatenate(xs).astype(np.float32),
            "adj_off": np.asarray(aoff, dtype=np.int64),
            "adj_ij": np.concatenate(ij).astype(np.int32) if ij else np.zeros((0, 2), np.int32),
            "adj_w": np.concatenate(w).astype(np.float32),
            "targets": np.stack(ts).astype(np.float32),
        }
        for k, v in data.items():
            np.save(os.path.join(path, k + ".npy"), v, allow_pickle=False)
        meta = {"format": FORMAT, "version": VERSION, "graphs": len(ts), "features": int(f), "targets": int(n_t),
                "nodes": int(offs[-1]), "adj_nnz": int(aoff[-1])}
        with open(os.path.join(path, "meta.json"), "w") as fh:
            json.dump(meta, fh, indent=1)
        return GraphPack(path)

    def __len__(self):
        return len(self.node_off) - 1

    def graph(self, i):
        """(x (n, f), A (n, n), t (n_t,)) CPU float32 tensors of graph i."""
        n0, n1 = int(self.node_off[i]), int(self.node_off[i + 1])
        a0, a1 = int(self.adj_off[i]), int(self.adj_off[i + 1])
        x = torch.from_numpy(np.array(self.x[n0:n1]))
        a = torch.zeros(n1 - n0, n1 - n0)
        if a1 > a0:
            ij = torch.from_numpy(np.array(self.adj_ij[a0:a1], dtype=np.int64))
            a[ij[:, 0], ij[:, 1]] = torch.from_numpy(np.array(self.adj_w[a0:a1]))
        t = torch.from_numpy(np.array(self.targets[i]))
        return x, a, t

    def instances(self, idx, J=1, dual=True):
        """Reference 7-tuples (x, A, t, W, WL, Pm, Pd) -- or (x, A, t, W) with dual=False -- for the
        indices, operators from the native builder (functions.operators.graph_operators)."""
        from functions.operators import graph_operators
        out = []
        for i in idx:
            x, a, t = self.graph(i)
            ops = graph_operators([x, a], J, dual)
            out.append([x, a, t, *(ops if dual else [ops])])
        return out

    def batches(self, idx, batch_size, task, J=1, dual=True, device="cuda", dense=False):
        """Yield one batch per `batch_size` consecutive indices of `idx`: a CsrBatch (the executor's
        layout, built natively from the mapped arrays) or, with dense=True, the reference's
        prepare_batch 11-tuple."""
        from functions.batching import prepare_batch
        from .csr import CsrBatch
        idx = list(idx)
        for b0 in range(0, len(idx), batch_size):
            part = idx[b0:b0 + batch_size]
            if dense:
                yield prepare_batch(self.instances(part, J, dual), task, J)
                continue
            graphs = [self.graph(i) for i in part]
            targets = torch.tensor([float(t[task]) for _, _, t in graphs], dtype=torch.float32)
            yield CsrBatch([(x, a) for x, a, _ in graphs], J=J, dual=dual, targets=targets, device=device)


# ---------------------------------------------------------------- QM9 .xyz
XYZ_PROPS = ("tag", "ident", "A", "B", "C", "mu", "alpha", "homo", "lumo", "gap", "r2", "zpve", "U0", "U", "H", "G",
             "Cv")
# molecule_to_instance's task order (preprocessing/preprocessing.py:44-57); task 8 is the last frequency
TARGETS = ("alpha", "Cv", "G", "gap", "H", "homo", "lumo", "mu", "freq_last", "r2", "U", "U0", "zpve")


def _num(s):
    # QM9 writes some exponents as '*^' (and '.*^'), preprocessing.py:189-190
    return float(s.replace(".*^", "e").replace("*^", "e"))


def read_xyz(path_or_text):
    """Parse one QM9 `.xyz` file (preprocessing/preprocessing.py:174-236, minus the rdkit part):
    dict with Na, the 17 header properties, atoms [(symbol, (x, y, z), partial charge)], freq
    and smiles."""
    text = path_or_text
    if "\n" not in path_or_text and os.path.exists(path_or_text):
        with open(path_or_text) as fh:
            text = fh.read()
    lines = text.splitlines()
    na = int(lines[0])
    prop = lines[1].split()
    mol = {"Na": na, "tag": prop[0], "ident": int(prop[1])}
    for k, v in zip(XYZ_PROPS[2:], prop[2:]):
        mol[k] = _num(v)
    atoms = []
    for i in range(na):
        p = lines[2 + i].split()
        atoms.append((p[0], tuple(_num(c) for c in p[1:4]), _num(p[4])))
    mol["atoms"] = atoms
    mol["freq"] = [_num(v) for v in lines[2 + na].split()]
    mol["smiles"] = lines[3 + na].split()[0]
    return mol


def molecule_targets(mol):
    """The 13-vector `task` of molecule_to_instance (preprocessing/preprocessing.py:44-57)."""
    t = torch.zeros(13)
    for k, name in enumerate(TARGETS):
        t[k] = float(mol["freq"][-1]) if name == "freq_last" else mol[name]
    return t


def atom_one_hot(symbols):
    """(n, 5) one-hot over H, C, N, O, other (preprocessing/preprocessing.py:60-77)."""
    col = {"H": 0, "C": 1, "N": 2, "O": 3}
    x = torch.zeros(len(symbols), 5)
    for i, s in enumerate(symbols):
        x[i, col.get(s, 4)] = 1.0
    return x


def molecule_instance(mol, bonds, spatial=False, charge=False):
    """(x, A, t) of molecule_to_instance (preprocessing/preprocessing.py:25-94) for atoms in the
    file's order and bonds = [(i, j, order)] supplied by the caller (the reference gets them, and
    its atom order, from rdkit).  Keeps the reference's indentation quirk: the spatial / charge
    columns are written for the LAST atom only (preprocessing.py:79-86)."""
    width = 5 + (3 if spatial else 0) + (1 if charge else 0)
    x = torch.zeros(mol["Na"], width)
    x[:, :5] = atom_one_hot([a[0] for a in mol["atoms"]])
    i = mol["Na"] - 1
    if spatial:
        x[i, 5:8] = torch.tensor(mol["atoms"][i][1])
        if charge:
            x[i, 8] = mol["atoms"][i][2]
    elif charge:
        x[i, 5] = mol["atoms"][i][2]
    a = torch.zeros(mol["Na"], mol["Na"])
    for u, v, order in bonds:
        a[u, v] = order
        a[v, u] = order
    return x, a, molecule_targets(mol)
