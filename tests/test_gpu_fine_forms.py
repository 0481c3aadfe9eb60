"""The level-0 kernel's launch forms give the same z bit for bit: the default
(one block per wave, two-wave workgroups dealt to the XCDs in contiguous
chunks), the inverses split into a default-policy and a nontemporal launch
(MAS_RESIDENT_SPLIT), and the per-size cache policy forced either way
(MAS_INV_RESIDENT), on cloth and tet meshes, an odd vertex count and the
one-level case (k_apply.hip launch_fine)."""
import numpy as np
import pytest

from conftest import cloth, tet

pytestmark = pytest.mark.gpu

FORMS = [{}, {"MAS_RESIDENT_SPLIT": "7"}, {"MAS_INV_RESIDENT": "0"}, {"MAS_INV_RESIDENT": "1"}]


@pytest.mark.parametrize("kind,W,L", [("cloth", 100, 3), ("cloth", 256, 4), ("cloth", 33, 1), ("tet", 16, 4)])
def test_fine_forms_bitwise(kind, W, L, monkeypatch):
    import torch
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 31)).cuda()
    out = []
    for env in FORMS:
        for k in ("MAS_RESIDENT_SPLIT", "MAS_INV_RESIDENT"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        P = mas_amd.from_mesh(mesh, max_levels=L)
        z = torch.zeros_like(r)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        for _ in range(2):  # the second apply over the first one's z
            P.PreconditioningDevice(z, r, s.cuda_stream)
        s.synchronize()
        out.append(z.cpu().numpy())
    for env, z in zip(FORMS[1:], out[1:]):
        assert np.array_equal(z.view(np.uint32), out[0].view(np.uint32)), env
