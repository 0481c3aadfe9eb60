"""Hash of sampled block inverses of a prepared config (bitwise A/B of two
library builds: run once per MAS_LIB_NAME and compare the printed digests)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/python"))
import mas_amd  # noqa: E402
from mas_amd import meshgen  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts)
nb = P.info()["num_blocks"]
h = hashlib.sha256()
for b in list(range(0, nb, max(1, nb // 2000))) + [nb - 1]:
    h.update(P.block_inverse(b).tobytes())
z = P.Preconditioning(None, meshgen.residual(mesh.nV, 7))
h2 = hashlib.sha256(z.tobytes()).hexdigest()[:16]
print(cfg_name, "inverses", h.hexdigest()[:16], "z", h2, flush=True)
