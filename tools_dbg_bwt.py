import sys, numpy as np
sys.path.insert(0, "high-order-entropy-compressed-suffix-array_amd"); sys.path.insert(0, ".")
import hkcsa
from oracle import oracle
for n in [20001, (1 << 22) + 1]:
    text = oracle.synth_text(n, b"ACGT", seed=21)
    dev = hkcsa.DeviceIndex.from_bytes(text.tobytes(), device=0)
    dev.build_sa(); sa = dev.sa(); b = dev.bwt(); w = oracle.bwt(text, sa)
    bad = np.nonzero(b != w)[0]
    print(n, "mismatches", len(bad), dev.build_info()[:10])
    for i in bad[:12]:
        print("  i", i, "sa", sa[i], "got", chr(b[i]), "want", chr(w[i]))
