import sys, numpy as np
sys.path.insert(0, '.')
from yalm_amd import runtime as rt
np.set_printoptions(linewidth=200, precision=3, suppress=True)
n, d = 256, 16
x = np.arange(n, dtype=np.float32)
w = np.zeros((d, n), np.float32)
for i in range(d): w[i, i] = 1
print("ident f32", rt.matmul(x, w, 0))
w = np.ones((d, n), np.float32)
print("ones f32", rt.matmul(x, w, 0), x.sum())
w = np.zeros((d, n), np.float32); w[:, 0] = 1
print("col0", rt.matmul(np.ones(n, np.float32), w, 0))
w = np.zeros((d, n), np.float32); w[3, :] = 1
print("row3", rt.matmul(np.ones(n, np.float32), w, 0))
w = np.zeros((d, n), np.float16)
for i in range(d): w[i, i*3] = 1
print("ident f16", rt.matmul(x, w, 1))
