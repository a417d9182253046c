import sys, json, time
sys.path.insert(0, '/root/repo')
import numpy as np
from leanfe_amd import synth, inference
from leanfe_amd._lib import Engine
n, k, L = 50_000_000, 10, [100_000, 1_000]
beta = synth.betas(k)
with Engine(0) as eng:
    eng.synth_load_codes(n, k, L, seed=12345)
    for rep in range(3):
        eng.profile(True)
        n_obs, dims, card = eng.drop_singletons()
        eng.stream_synth_pass(1, k, L, beta, chunk_rows=n, seed=12345)
        it, _ = eng.demean(sorted(range(2), key=lambda i: card[i]), 1e-6, 50, check_from=3)
        G = eng.gram()
        XtX, Xty = inference.split_gram(G)
        bf, XtX_inv = inference.solve_normal(XtX, Xty)
        out = eng.stream_synth_pass(2, k, L, beta, chunk_rows=n, seed=12345, beta_full=bf)
        ks = eng.kernel_stats()
    print(json.dumps({kk: [round(v[0], 4), v[1]] for kk, v in ks.items()}))
