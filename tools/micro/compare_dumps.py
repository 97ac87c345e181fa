"""Compare two render_dump.py outputs bit for bit."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
ok = True
for k in a.files:
    same = np.array_equal(a[k], b[k])
    ok &= same
    print(k, "identical" if same else f"DIFFERENT ({int((a[k] != b[k]).sum())} words)")
sys.exit(0 if ok else 1)
