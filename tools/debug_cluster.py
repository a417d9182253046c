"""Debug: per-array cluster meats from the engine vs NumPy on the xlang_cl2 fixture."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from golden_util import load
from oracle import altproj
from leanfe_amd import frame, inference
from leanfe_amd._lib import Engine

meta, data, exp = load("xlang_cl2")
r = altproj.fit(data, meta["y"], meta["xs"], meta["fes"], vcov="cluster", cluster_cols=meta["cluster_cols"])
X = r["demeaned"][1:].T; res = r["resid"]; U = X * res[:, None]
cols = [np.asarray(data[meta["y"]], float)] + [np.asarray(data[x], float) for x in meta["xs"]]
codes, lv = zip(*[frame.factorize(data[f]) for f in meta["fes"]])
eng = Engine(0)
eng.load(cols, list(codes), list(lv))
n, dims, card = eng.drop_singletons()
it, _ = eng.demean([1, 0], 1e-6, 50, 3)
G = eng.gram(); XtX, Xty = inference.split_gram(G); bf, inv = inference.solve_normal(XtX, Xty)
print("beta dev", np.max(np.abs(bf[1:] - r["beta"])))
stats, _ = eng.resid(bf, keep_scores=True)
print("rss", stats[1], np.sum(res ** 2))
dm = eng.copy_demeaned(n)
print("demeaned dev", np.max(np.abs(dm[1:].T - X)))
c1, g1 = frame.factorize(data["cluster"]); c2, g2 = frame.factorize(data["fe2"])
c12, g12 = frame.intersect([c1, c2], [g1, g2])
for arrs, lvs in [([c1], [g1]), ([c2], [g2]), ([c12], [g12]), ([c1, c2, c12], [g1, g2, g12])]:
    eng.load_clusters(arrs, lvs)
    meats, Gs = eng.cluster_meat()
    for a, m, g in zip(arrs, meats, Gs):
        S = np.zeros((a.max() + 1, 3)); np.add.at(S, a, U)
        ref = S.T @ S
        print(len(arrs), "G", g, "meat rel dev", np.max(np.abs(m - ref)) / np.max(np.abs(ref)))
