import sys, os, ctypes as C
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("icp-4dradar_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import icp4r, oracle
L = icp4r.load(); OL = oracle.lib()
rng = np.random.default_rng(0)
k = 2000
S = rng.normal(0, 100, (k, 9)).astype(np.float32)
S[:1000] = (np.eye(3).ravel()[None, :] * 500 + rng.normal(0, 1, (1000, 9))).astype(np.float32)
ctx = icp4r.Context(0, plan=icp4r.env_plan())
Rg = np.zeros((k, 9), np.float32)
rc = L.icp4r__test_rot_f32(ctx.handle, C.c_void_p(S.ctypes.data), C.c_void_p(Rg.ctypes.data), k)
assert rc == 0, rc
Ro = np.zeros((k, 9), np.float32)
for i in range(k):
    OL.oracle_rot_f32(C.c_void_p(S[i].ctypes.data), C.c_void_p(Ro[i].ctypes.data))
diff = (Rg.view(np.int32) != Ro.view(np.int32)).any(1)
print("mismatching matrices:", int(diff.sum()), "of", k)
i = int(np.argmax(diff)) if diff.any() else None
if i is not None:
    print(S[i]); print(Rg[i]); print(Ro[i])
