"""Timeline of the one-launch coarse kernel (k_coarse1.hip) from the probe build
(make -C <pkg> probe).  usage: python scripts/dev/probe_coarse1.py CONFIG
Per role, the spread of wave starts and each stamp relative to the first start (us)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
os.environ.setdefault("MAS_LIB_NAME", "libmas_amd_probe.so")
os.environ.setdefault("MAS_COARSE_MODE", "3")
import numpy as np
import torch
import mas_amd
from mas_amd import meshgen

name = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
mesh, cfg = meshgen.build_config(name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts)
lib = P._L
lib.mas_probe1_dump.argtypes = [ctypes.c_void_p, ctypes.c_int]
r = torch.from_numpy(meshgen.residual(mesh.nV, 1)).cuda()
z = torch.zeros_like(r)
for it in range(20):
    lib.mas_probe1_clear()
    torch.cuda.synchronize()
    P.PreconditioningDevice(z, r, 0)
    torch.cuda.synchronize()
buf = np.zeros(3 * 8192 * 8, np.uint64)
lib.mas_probe1_dump(buf.ctypes.data, buf.size)
buf = buf.reshape(3, 8192, 8).astype(np.int64)
t0 = buf[buf > 0].min()
print(name, "levels", P.info()["level_size"].tolist())
labels = {0: ["start", "first prefix / R2 polled", "fold end", "R3 published"],
          1: ["start", "staged", "R1/R2 published", "Z1 stored"],
          2: ["start", "R polled", "Z stored"]}
names = {0: "level-3 fold waves", 1: "bank waves", 2: "level-2 solve waves", 3: "level-3 solve waves"}
nb2 = (int(P.info()["level_size"][2][0]) + 31) // 32  # solve-wave slots: level 2 first, then level 3
for kind in (0, 1, 2, 3):
    b = buf[min(kind, 2)]
    if kind >= 2:
        b = b[:nb2] if kind == 2 else b[nb2:]
    live = b[:, 0] > 0
    if not live.any():
        continue
    b = b[live]
    print(f"{names[kind]}: {len(b)}")
    for s, lab in enumerate(labels[min(kind, 2)]):
        m = b[:, s] > 0
        if not m.any():
            continue
        e = (b[m, s] - t0) / 100
        print(f"  {s} {lab:18s} n={m.sum():5d}  at {e.min():7.2f} / med {np.median(e):7.2f} / max {e.max():7.2f} us")
