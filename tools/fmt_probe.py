# Storage formats (sss_hip_level_info a_format / r_format / p_format bits) of each level of a 7-pt hierarchy on the GPU:
#   python tools/fmt_probe.py 64
import sys; sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import amg_amd as A
from conftest import build_hierarchy, quiet_ctx
H = build_hierarchy(A.generate(7, int(sys.argv[1])), quiet_ctx)
D = A.DeviceHierarchy(H, smoother="hybrid", coarse="direct", device=0, sum_order=1)
for l in range(H.num_levels - 1):
    i = D.level_info(l); print(l, i.a_format, i.r_format, i.p_format)
