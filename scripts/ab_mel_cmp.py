import sys
import numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in a.files:
    d = np.abs(a[k] - b[k])
    print(k, a[k].shape, "bit-equal" if np.array_equal(a[k], b[k]) else "max|d| %.3e rel %.3e" % (d.max(), d.max() / np.abs(a[k]).max()))
