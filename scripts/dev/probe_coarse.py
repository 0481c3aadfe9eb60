"""Timeline of the coarse kernels from the diagnostic stamp build
(make -C <pkg> probe; MAS_LIB_NAME=libmas_amd_probe.so python scripts/dev/probe_coarse.py [W] [L]).
Prints, per kernel, the spread of wave starts and the median/max of each
stamp-to-stamp segment (us), relative to the kernel's first wave start."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
os.environ.setdefault("MAS_LIB_NAME", "libmas_amd_probe.so")
import numpy as np
import torch
import mas_amd
from mas_amd import meshgen

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
L = int(sys.argv[2]) if len(sys.argv) > 2 else 4
mesh = meshgen.cloth_grid(W)
contacts = meshgen.vf_contacts(mesh, 100_000 if W == 1024 else 0, seed=3) if W == 1024 else None
P = mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts)
lib = P._L
lib.mas_probe_dump.argtypes = [ctypes.c_void_p, ctypes.c_int]
r = torch.from_numpy(meshgen.residual(mesh.nV, 1)).cuda()
z = torch.zeros_like(r)
for it in range(30):
    lib.mas_probe_clear()
    torch.cuda.synchronize()
    P.PreconditioningDevice(z, r, 0)
    torch.cuda.synchronize()
buf = np.zeros(2 * 4096 * 8, np.uint64)
lib.mas_probe_dump(buf.ctypes.data, buf.size)
buf = buf.reshape(2, 4096, 8).astype(np.int64)
# deep workgroups (k_solve123 waves 0 .. 4 * n3 - 1): start, list landed (stamp 5), fold end, arrival
n3 = int(P.info()["level_size"].reshape(-1)[6]) if L >= 4 else 0
if n3:
    d = buf[1, :4 * n3].copy()
    t0d = d[:, 0][d[:, 0] > 0].min()
    rel = lambda x: (x[x > 0] - t0d) / 100
    print(f"deep: {n3} nodes; list landed (wave 0) {np.median(rel(d[0::4, 5])):.2f} us median, max {rel(d[0::4, 5]).max():.2f};"
          f" fold end {rel(d[0::4, 2]).max():.2f}; arrivals {rel(d[0::4, 3]).max():.2f}; solve {rel(d[:, 4]).max() if (d[:, 4] > 0).any() else 0:.2f}")
info = P.info()
print("levels", info["level_size"].tolist())
t0 = buf[buf > 0].min()
for k, name in enumerate(["k_restrict12", "k_solve123"]):
    b = buf[k]
    live = b[:, 0] > 0
    b = b[live]
    idx = np.flatnonzero(live)
    print(f"{name}: {len(b)} waves, starts {(b[:, 0].min() - t0) / 100:.2f} .. {(b[:, 0].max() - t0) / 100:.2f} us")
    for s in range(1, 7):
        m = b[:, s] > 0
        if not m.any():
            continue
        d = (b[m, s] - b[m, s - 1]) / 100
        e = (b[m, s] - t0) / 100
        print(f"  seg {s - 1}->{s}: n={m.sum():5d} median {np.median(d):6.2f} max {d.max():6.2f}  stamp {s} at {e.min():6.2f}..{e.max():6.2f} us")
