"""Debug dump of the fold waves (probe build): len, banks, entries folded, polls."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests")); sys.path.insert(0, os.path.join(REPO, "oracle"))
os.environ.setdefault("MAS_LIB_NAME", "libmas_amd_probe.so")
import numpy as np, torch, mas_amd
from mas_amd import meshgen
W, L = int(sys.argv[1]), int(sys.argv[2])
mesh = meshgen.cloth_grid(W)
out = {}
for mode in ("2", "3"):
    os.environ["MAS_COARSE_MODE"] = mode
    P = mas_amd.from_mesh(mesh, max_levels=L)
    lib = P._L
    lib.mas_probe1_dump.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.mas_probe1_clear()
    r = torch.from_numpy(meshgen.residual(mesh.nV, 40)).cuda(); z = torch.zeros_like(r)
    torch.cuda.synchronize(); P.PreconditioningDevice(z, r, 0); torch.cuda.synchronize()
    out[mode] = P.coarse_residual()
    if mode == "3":
        buf = np.zeros(2 * 8192 * 8, np.uint64); lib.mas_probe1_dump(buf.ctypes.data, buf.size)
        b = buf.reshape(2, 8192, 8)
        info = P.info(); print("levels", info["level_size"].tolist())
        n3 = int(info["level_size"][3][0])
        for T in range(n3 + 2):
            print(T, "len", int(b[0, T, 5]), "nb", int(b[0, T, 6]) & 0xffff, "ready", int(b[0, T, 6]) >> 16,
                  "e", int(b[0, T, 7]) & 0xfffff, "polls", (int(b[0, T, 7]) >> 20) & 0xfffff, "E1", int(b[0, T, 7]) >> 40)
ls = P.info()["level_size"]; b1 = int(ls[1][1])
for l in range(1, min(P.info()["num_levels"], 4)):
    beg, cnt = int(ls[l][1]) - b1, int(ls[l][0])
    d = np.abs(out["2"][beg:beg + cnt] - out["3"][beg:beg + cnt]).max()
    print("level", l, "max diff", d)
    if l == 3: print(out["2"][beg:beg + cnt], out["3"][beg:beg + cnt])
