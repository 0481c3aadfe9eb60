"""Write tests/golden/cloth12_L0.masblob: the blob of Allocate + Prepare of the
12x12 cloth grid (default levels), produced by the HIP path on an MI355X.
Run on the GPU box: python scripts/make_golden_blob.py gpurun_out/cloth12_L0.masblob"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import mas_amd  # noqa: E402
from mas_amd import meshgen  # noqa: E402

mesh = meshgen.cloth_grid(12)
P = mas_amd.from_mesh(mesh, max_levels=0)
blob = P.save_blob()
blob.tofile(sys.argv[1])
print(sys.argv[1], blob.nbytes, "bytes")
