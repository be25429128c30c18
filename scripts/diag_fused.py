import sys, numpy as np
sys.path.insert(0, "q-learning_amd"); sys.path.insert(0, "tests")
import qlx
import ctypes as C
from test_gpu_qnet import rand_states
B = 1024
fused, plain = qlx.DeepQLearningModel(seed=21), qlx.DeepQLearningModel(seed=21)
x = rand_states(B, 3, sparse=True)
rng = np.random.default_rng(2)
a = rng.integers(0, 3, B).astype(np.uint8)
y = rng.normal(0, 1, B).astype(np.float32)
L = qlx.lib()
for it in range(6):
    nf = np.zeros(10, np.float32); lf = C.c_float()
    xs = np.ascontiguousarray(x); 
    L.qlx_model_train(fused.h, qlx._p(xs), qlx._p(a), qlx._p(y), B, C.byref(lf), None, qlx._p(nf))
    lp, g, npn = plain.train(x, a, y, want_grads=True)
    print("it", it, "loss", lf.value, lp, "norms fused", nf[6:8], "plain", npn[6:8])
    for v in (6, 7):
        for which in range(3):
            d = fused.get(v, which) - plain.get(v, which)
            nz = np.count_nonzero(d)
            if nz:
                print("  var", v, "which", which, "ndiff", nz, "maxabs", np.abs(d).max(), "first idx", np.flatnonzero(d.ravel())[:8])
