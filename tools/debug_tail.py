"""Debug probe for the in-slot nonce/tag path (read_tail/write_tail) at every L % 4."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import oracle as O
from quantum_amd import batch
from quantum_amd.crypto import Context
ctx = Context(0, 4)
key = bytes(range(32)); ctx.set_key(0, key)
nonce = bytes(range(100, 112))
for L in (0, 1, 2, 3, 4, 5, 17, 18, 19, 1350):
    for pz in (True, False):
        stride = batch.slot_stride(L)
        h = np.zeros(stride, np.uint8); h[:4] = [10, 99, 0, 1]
        pt = bytes(L) if pz else bytes((7 * i + 1) & 0xff for i in range(L))
        h[4:4 + L] = np.frombuffer(pt, np.uint8)
        h[4 + L + 16:4 + L + 28] = np.frombuffer(nonce, np.uint8)
        arena = torch.from_numpy(h.copy()).cuda()
        batch.seal_uniform(ctx, arena, stride, 1, L, 0, None, aad_len=4)
        got = arena.cpu().numpy().tobytes()[4:4 + L + 28]
        ct, tag = O.gcm_seal(key, nonce, bytes(h[:4]), pt)
        want = ct + tag + nonce
        # also the explicit-nonce path for the same input
        h2 = h.copy(); a2 = torch.from_numpy(h2).cuda()
        non = torch.from_numpy(np.frombuffer(nonce, np.uint8).copy()).cuda()
        batch.seal_uniform(ctx, a2, stride, 1, L, 0, non, aad_len=4)
        got2 = a2.cpu().numpy().tobytes()[4:4 + L + 28]
        print(f"L={L:4d} zero_pt={pz} slot_nonce_ok={got == want} array_nonce_ok={got2 == want} "
              f"ct_ok={got[:L] == ct} tag_ok={got[L:L+16] == tag} nonce_ok={got[L+16:] == nonce}")
        if got != want and L < 20:
            print("   got ", got.hex()); print("   want", want.hex()); print("   arr ", got2.hex())
