"""CPU check of the device DBSCAN merge algorithm (union-find over labels with zero-class nodes,
k_dbscan_merge) against a literal transcription of DBSCAN_EdgeFeature's merge loop
(featureAssociation.cpp:1342-1386), on random neighbourhood relations including the quirks:
non-reflexive rows (eps(i,i) NaN), empty rows, asymmetric eps."""
import numpy as np


def reference_merge(adj):
    M = adj.shape[0]
    cluster = [0] * M
    label = 0
    for i in range(M):
        cluster[i] = 0
        in_idx = [j for j in range(M) if adj[i, j]]
        in_labels = [cluster[j] for j in in_idx]
        nz = [cluster[j] for j in in_idx if cluster[j] != 0]
        min_label = min(nz) if nz else 999999999
        if min_label <= label:
            L = set(in_labels)
            for j in range(M):
                if cluster[j] in L:
                    cluster[j] = min_label
            for j in in_idx:
                cluster[j] = min_label
        else:
            label += 1
            for j in in_idx:
                cluster[j] = label
    return cluster


def uf_merge(adj):
    """Restatement of the device algorithm."""
    M = adj.shape[0]
    Z0 = M + 1
    parent = list(range(2 * M + 3))
    raw = [Z0] * M
    live = [Z0]
    label = 0

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for i in range(M):
        zi = M + 2 + i
        raw[i] = zi
        nbrs = np.nonzero(adj[i])[0].tolist()
        roots = [find(raw[j]) for j in nbrs]
        eff = [0 if r > M else r for r in roots]
        nz = [e for e in eff if e != 0]
        min_label = min(nz) if nz else 999999999
        zero_present = any(e == 0 for e in eff)
        i_in = bool(adj[i, i])
        if min_label <= label:
            for r in roots:
                if r <= M and r != min_label:
                    parent[r] = min_label
            if zero_present:
                for z in live + [zi]:
                    parent[find(z)] = min_label if find(z) > M else parent[find(z)]
                live = []
            elif not i_in:
                live.append(zi)
            for j in nbrs:
                raw[j] = min_label
        else:
            label += 1
            for j in nbrs:
                raw[j] = label
            if not i_in:
                live.append(zi)
    out = []
    for j in range(M):
        r = find(raw[j])
        out.append(0 if r > M else r)
    return out


def test_uf_dbscan_matches_reference_loop():
    rng = np.random.default_rng(7)
    for trial in range(400):
        M = int(rng.integers(0, 40))
        p = rng.uniform(0.02, 0.3)
        adj = rng.random((M, M)) < p
        if trial % 3 == 0:  # symmetric, reflexive (the common geometric case)
            adj = adj | adj.T
            np.fill_diagonal(adj, True)
        elif trial % 3 == 1:
            np.fill_diagonal(adj, rng.random(M) < 0.8)
        assert uf_merge(adj) == reference_merge(adj), (trial, M)
