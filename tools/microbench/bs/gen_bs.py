"""Generates the bitsliced AES S-box for gfx950 as v_bitop3_b32 (3-input) gates.

Layout: q[j] = bit j (LSB = 0) of the byte, 32 slots per 32-bit word.
Circuit: the Boyar-Peralta 113-gate S-box (top linear layer, 32 ANDs, bottom linear layer).  Both
linear layers are re-derived as XOR3/XOR2 straight-line programs (slp3.py); the whole circuit is
then greedily merged (a fanout-1 gate folds into its consumer when the result has <= 3 inputs) and
checked on all 256 inputs before anything is emitted.
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from bp_circuit import lines, SB  # noqa: E402
from slp3 import search  # noqa: E402

XOR = lambda a, b: a ^ b  # noqa: E731
AND = lambda a, b: a & b  # noqa: E731


def parse():
    out = []
    for l in lines:
        d, e = l.split(" = ")
        a, op, neg, b = re.match(r"(\w+) ([&^]) (~?)(\w+)", e).groups()
        out.append((d, a, op, bool(neg), b))
    return out


def build_circuit(trials=60):
    g = parse()
    # linear forms of the top layer over x0..x7 and of the bottom layer over z0..z17
    xf = {f"x{i}": 1 << i for i in range(8)}
    zf = {f"z{i}": 1 << i for i in range(18)}
    zneg = {}
    for d, a, op, neg, b in g:
        if op == "^" and a in xf and b in xf and not neg:
            xf[d] = xf[a] ^ xf[b]
        if op == "^" and a in zf and b in zf:
            zf[d] = zf[a] ^ zf[b]
            zneg[d] = zneg.get(a, 0) ^ zneg.get(b, 0) ^ int(neg)
    ys = {d: v for d, v in xf.items() if d.startswith("y")}
    _, top = search({f"x{i}": 1 << i for i in range(8)}, ys, trials=trials, seed=11)
    outs = {f"s{i}": zf[f"s{i}"] for i in range(8)}
    _, bot = search({f"z{i}": 1 << i for i in range(18)}, outs, trials=trials, seed=12)
    # nodes: name -> (inputs, fn, expr)
    nodes, order = {}, []

    def add(name, ins, fn, expr):
        nodes[name] = (ins, fn, expr)
        order.append(name)

    for name, ops in top:
        assert len(ops) > 1
        if len(ops) == 2:
            add(name, ops, XOR, f"({ops[0]} ^ {ops[1]})")
        else:
            add(name, ops, lambda a, b, c: a ^ b ^ c, f"({ops[0]} ^ {ops[1]} ^ {ops[2]})")
    for d, a, op, neg, b in g:
        if d.startswith("y") or d in ("t0", "t1") or (op == "^" and a in zf and b in zf):
            continue
        if d.startswith("s"):
            continue
        if op == "&":
            add(d, [a, b], AND, f"({a} & {b})")
        else:
            assert not neg
            add(d, [a, b], XOR, f"({a} ^ {b})")
    # bottom: helper names must not clash with the top's
    ren, const = {}, {}
    for name, ops in bot:
        nn = ("b" + name) if name.startswith("h") else name
        ren[name] = nn
        ops = [ren.get(o, o) for o in ops]
        # the output complements (BP's XNORs) fold into each target's gate, net of the constants
        # its operands already carry
        carried = 0
        for o in ops:
            carried ^= const.get(o, 0)
        want = zneg.get(name, 0) if name.startswith("s") else carried
        inv = want ^ carried
        const[nn] = want
        if len(ops) == 2:
            fn = (lambda a, b: 1 ^ a ^ b) if inv else XOR
            add(nn, ops, fn, f"({'~' if inv else ''}({ops[0]} ^ {ops[1]}))")
        else:
            fn = (lambda a, b, c: 1 ^ a ^ b ^ c) if inv else (lambda a, b, c: a ^ b ^ c)
            add(nn, ops, fn, f"({'~' if inv else ''}({ops[0]} ^ {ops[1]} ^ {ops[2]}))")
    return nodes, order


def merge(nodes, order):
    outputs = {f"s{i}" for i in range(8)}
    changed = True
    while changed:
        changed = False
        fo = {}
        for d, (ins, _, _) in nodes.items():
            for i in ins:
                fo[i] = fo.get(i, 0) + 1
        for d in order:
            if d not in nodes:
                continue
            ins, f, ex = nodes[d]
            for i in list(ins):
                if i in nodes and fo.get(i, 0) == 1 and i not in outputs:
                    iins, ifn, iex = nodes[i]
                    new = []
                    for x in ins:
                        for y in (iins if x == i else [x]):
                            if y not in new:
                                new.append(y)
                    if len(new) <= 3:
                        def mk(ins=ins, f=f, i=i, iins=iins, ifn=ifn, new=new):
                            def gfn(*vals):
                                env = dict(zip(new, vals))
                                env[i] = ifn(*[env[y] for y in iins])
                                return f(*[env[x] for x in ins])
                            return gfn
                        nodes[d] = (new, mk(), re.sub(r"\b%s\b" % i, iex, ex))
                        del nodes[i]
                        changed = True
                        break
            if changed:
                break
    return [d for d in order if d in nodes]


def check(nodes, topo):
    def run(x):
        env = {f"x{i}": (x >> (7 - i)) & 1 for i in range(8)}
        for d in topo:
            ins, f, _ = nodes[d]
            env[d] = f(*[env[i] for i in ins]) & 1
        return sum(env[f"s{i}"] << (7 - i) for i in range(8))

    bad = [x for x in range(256) if run(x) != SB[x]]
    assert not bad, f"S-box circuit wrong on {len(bad)} inputs"


def emit(nodes, topo):
    out = [
        "// Generated by tools/microbench/bs/gen_bs.py: Boyar-Peralta AES S-box, linear layers",
        f"// re-derived as XOR3 programs, merged into {len(topo)} v_bitop3_b32 / 2-input gates.",
        "// In/out: q[j] = bit j (LSB 0) of the byte, 32 slots per word.",
        "__device__ __forceinline__ void bs_sbox(uint32_t *q) {",
    ]
    for i in range(8):
        out.append(f"    const uint32_t x{i} = q[{7 - i}];")
    for d in topo:
        ins, f, ex = nodes[d]
        if len(ins) <= 2 and "~" not in ex:
            out.append(f"    const uint32_t {d} = {ex};")
        else:
            ins3 = ins + [ins[-1]] * (3 - len(ins))
            tt = 0
            for bit in range(8):  # v_bitop3 truth table: f on the canonical bytes S0=0xf0, S1=0xcc, S2=0xaa
                vals = [(0xF0 >> bit) & 1, (0xCC >> bit) & 1, (0xAA >> bit) & 1][: len(ins)]
                tt |= (f(*vals) & 1) << bit
            out.append(f"    const uint32_t {d} = __builtin_amdgcn_bitop3_b32({ins3[0]}, {ins3[1]}, {ins3[2]}, 0x{tt:02x});"
                       f"  // {ex}")
    for i in range(8):
        out.append(f"    q[{7 - i}] = s{i};")
    out.append("}")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    trials = int(os.environ.get("TRIALS", "60"))
    nodes, order = build_circuit(trials)
    topo = merge(nodes, order)
    check(nodes, topo)
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "bs_sbox.inc")
    with open(dst, "w") as f:
        f.write(emit(nodes, topo))
    print("wrote", dst, len(topo), "gates")
