import numpy as np, glob, os, sys
a, b = sys.argv[1], sys.argv[2]
bad = 0
for f in sorted(glob.glob(os.path.join(a, "*.npy"))):
    x = np.load(f); y = np.load(os.path.join(b, os.path.basename(f)))
    same = np.array_equal(x.view(np.uint8), y.view(np.uint8))
    bad += not same
    print(os.path.basename(f), "identical" if same else f"DIFF max {np.abs(x - y).max()}")
print("all identical" if bad == 0 else f"{bad} differ")
