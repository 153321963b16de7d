"""Quick GPU check: parity vs oracle on mixed vectors + rough throughput."""
import hashlib, os, random, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import oracle
from fabric_amd import synth, _lib

N_ORDER = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
rng = random.Random(7)
keys = [synth.Key(11, i) for i in range(8)]
K, S, D, M = [], [], [], []
for i in range(600):
    k = keys[i % 8]
    msg = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 300)))
    d = hashlib.sha256(msg).digest()
    kind = i % 10
    sig = synth.sign(k, d)
    if kind == 1: sig = synth.sign(k, d, high_s=True)
    elif kind == 2: d = hashlib.sha256(msg + b"x").digest()
    elif kind == 3: sig = sig[:-1]
    elif kind == 4: sig = sig + b"\x00\x01"  # trailing garbage: valid in Go
    elif kind == 5:
        r, s = synth.sign_rs(k, d); sig = synth.der_encode(r + N_ORDER if r + N_ORDER < 2**256 else r, s)
    elif kind == 6: sig = b""
    K.append(k.pub if kind != 7 else k.qx + bytes(32)); S.append(sig); D.append(d); M.append(msg)
exp = np.array([oracle.verify_der(K[i][:32], K[i][32:], S[i], D[i]) for i in range(len(S))], np.uint8)
print("expected status histogram", np.bincount(exp))
eng = _lib.Engine(0)
st = eng.verify_batch(np.frombuffer(b"".join(K), np.uint8).reshape(-1, 64), S, np.frombuffer(b"".join(D), np.uint8).reshape(-1, 32))
bad = np.nonzero(st != exp)[0]
print("verify_batch mismatches:", len(bad), [(int(i), int(st[i]), int(exp[i])) for i in bad[:10]])
dg = eng.sha256_batch(M)
print("sha mismatches:", sum(bytes(dg[i]) != hashlib.sha256(M[i]).digest() for i in range(len(M))))
st2 = eng.verify_msgs(np.frombuffer(b"".join(K), np.uint8).reshape(-1, 64), M, S)
exp2 = np.array([oracle.identity_verify(K[i][:32], K[i][32:], M[i], S[i]) for i in range(len(S))], np.uint8)
print("verify_msgs mismatches:", int((st2 != exp2).sum()))
# throughput: n items over 16 keys
for n in [16384, 131072, 524288]:
    ks = [synth.Key(3, i) for i in range(16)]
    base_d = [hashlib.sha256(str(i).encode()).digest() for i in range(256)]
    base = [(ks[i % 16], base_d[i], synth.sign(ks[i % 16], base_d[i])) for i in range(256)]
    kk = np.frombuffer(b"".join(base[i % 256][0].pub for i in range(n)), np.uint8).reshape(-1, 64)
    dd = np.frombuffer(b"".join(base[i % 256][1] for i in range(n)), np.uint8).reshape(-1, 32)
    ss = [base[i % 256][2] for i in range(n)]
    eng.verify_batch(kk, ss, dd)
    t = time.time(); st = eng.verify_batch(kk, ss, dd); el = time.time() - t
    tm = eng.timing()
    print(f"n={n} valid={int((st==0).sum())} wall={el*1e3:.1f}ms verifies/s={n/el:,.0f} kernel: {tm} -> point-only {n/(tm['point_ms']/1e3):,.0f}/s")
