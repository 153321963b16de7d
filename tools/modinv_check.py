"""Verify tools/modinv_check output: x * inv == 1 mod n for every line."""
import subprocess
import sys

N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
out = subprocess.run([sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "100000"], capture_output=True,
                     text=True, check=True).stdout.split("\n")
bad = 0
for line in out:
    if not line:
        continue
    x, r = (int(v, 16) for v in line.split())
    if x * r % N != 1:
        bad += 1
        if bad < 5:
            print("BAD", hex(x), hex(r))
print(len(out) - 1, "inputs,", bad, "wrong")
sys.exit(1 if bad else 0)
