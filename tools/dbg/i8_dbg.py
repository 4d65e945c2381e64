import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
from biscotti_amd import _lib
from biscotti_amd.krum import Engine
from biscotti_amd.dist import unpack_upper
e = Engine(0)
def upper(X, mode):
    n, d = X.shape
    tX = torch.from_numpy(np.ascontiguousarray(X)).cuda()
    U = torch.empty(int(_lib.lib().bk_upper_elems(n)), dtype=torch.float64, device="cuda")
    e.set_f32_mode(mode)
    e.gram_upper_ptr(tX.data_ptr(), _lib.BK_F32, n, d, d, U.data_ptr())
    e.synchronize()
    e.set_f32_mode(0)
    return U.cpu().numpy()
for (n, d) in [(128, 64), (129, 64), (256, 128)]:
    rng = np.random.default_rng(1)
    X = rng.integers(-63, 64, size=(n, d)).astype(np.float32)
    Ue, Ui = upper(X, 0), upper(X, 3)
    Ge, Gi = unpack_upper(Ue, n), unpack_upper(Ui, n)
    G = X.astype(np.float64) @ X.astype(np.float64).T
    print(n, d, "exact==numpy", np.array_equal(Ge, G), "i8==numpy", np.array_equal(Gi, G),
          "trail", Ui[-4:], flush=True)
    bad = np.argwhere(Gi != G)
    print("  bad count", len(bad), "of", G.size, bad[:10].tolist(), flush=True)
    if len(bad):
        i, j = bad[0]
        print("  Gi", Gi[i, j], "G", G[i, j], "ratio", Gi[i, j] / G[i, j] if G[i, j] else None)
        # try hypotheses: G_i8 scaled, transposed, permuted rows
        r = Gi[:32, :32] / np.where(G[:32, :32] == 0, 1, G[:32, :32])
        print("  ratio block 0..4", np.round(r[:4, :4], 4).tolist())
        # which row of G does Gi row 0 match?
        for a in range(4):
            m = [bb for bb in range(min(n, 64)) if np.allclose(Gi[a, :64], G[bb, :64])]
            print("  Gi row", a, "matches G rows", m)
        print("  Gi[0,:8]", Gi[0, :8].tolist())
        print("  G [0,:8]", G[0, :8].tolist())
