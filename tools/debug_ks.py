"""Debug probe: seal zero plaintexts so ciphertext == keystream; compare with the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import oracle as O
from quantum_amd import batch
from quantum_amd.crypto import Context
ctx = Context(0, 4)
key = bytes(range(32)); ctx.set_key(0, key)
nonce = bytes(range(100, 112))
for L in (0, 1, 4, 15, 16, 17, 32, 48, 64):
    for aad_len in (0, 4):
        n = 1
        stride = batch.slot_stride(L)
        h = np.zeros(stride, np.uint8); h[:4] = [10, 99, 0, 1]
        arena = torch.from_numpy(h.copy()).cuda()
        non = torch.from_numpy(np.frombuffer(nonce, np.uint8).copy()).cuda()
        batch.seal_uniform(ctx, arena, stride, n, L, 0, non, aad_len=aad_len)
        got = arena.cpu().numpy().tobytes()[4:4 + L + 28]
        ct, tag = O.gcm_seal(key, nonce, bytes(h[:aad_len]), bytes(L))
        want = ct + tag + nonce
        blocks = [got[i:i+16] == want[i:i+16] for i in range(0, L, 16)]
        print(f"L={L:3d} aad={aad_len} ok={got == want} ct_blocks={blocks} tag_ok={got[L:L+16] == tag} nonce_ok={got[L+16:] == nonce}")
        if L in (1, 16) and got != want:
            print("   got ", got.hex()); print("   want", want.hex())
