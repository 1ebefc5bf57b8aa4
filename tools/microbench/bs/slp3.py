"""Randomised greedy search for short XOR3/XOR2 straight-line programs (the linear layers of the
bitsliced S-box).  Signals are GF(2) vectors as Python ints; one op = one v_bitop3_b32 (or v_xor)."""
import itertools
import random


def search(inputs, targets, trials=200, seed=1, cand_cap=6000):
    """inputs: {name: vec}; targets: {name: vec}. Returns (ops, program [(name, [operand names])])."""
    best = None
    rng = random.Random(seed)
    for _ in range(trials):
        avail = dict(inputs)
        prog = []
        byvec = {v: k for k, v in avail.items()}
        todo = {}
        for k, v in targets.items():
            if v in byvec:
                prog.append((k, [byvec[v]]))  # alias, no op
            else:
                todo[k] = v
        nh = 0
        while todo:
            names = list(avail)
            vecs = [avail[n] for n in names]
            pair = {}
            for i in range(len(names)):
                for j in range(i + 1, len(names)):
                    pair.setdefault(vecs[i] ^ vecs[j], (names[i], names[j]))
            single = {vecs[i]: names[i] for i in range(len(names))}
            done = False
            tk = list(todo)
            rng.shuffle(tk)
            for k in tk:
                v = todo[k]
                ops = None
                if v in pair:
                    ops = list(pair[v])
                else:
                    for i in range(len(names)):
                        r = v ^ vecs[i]
                        if r in pair and names[i] not in pair[r]:
                            ops = [names[i]] + list(pair[r])
                            break
                if ops:
                    prog.append((k, ops))
                    avail[k] = v
                    del todo[k]
                    done = True
                    break
            if done:
                continue
            cands = list(itertools.combinations(range(len(names)), 2)) + list(
                itertools.combinations(range(len(names)), 3))
            rng.shuffle(cands)
            best_h, best_s = None, -1
            for c in cands[:cand_cap]:
                h = 0
                for i in c:
                    h ^= vecs[i]
                if h == 0 or h in single:
                    continue
                s = 0
                for v in todo.values():
                    r = v ^ h
                    if r in pair or r in single:
                        s += 2
                    else:
                        for i in range(len(names)):
                            if (r ^ vecs[i]) in pair:
                                s += 1
                                break
                if s > best_s:
                    best_s, best_h = s, c
            h = 0
            for i in best_h:
                h ^= vecs[i]
            name = f"h{nh}"
            nh += 1
            prog.append((name, [names[i] for i in best_h]))
            avail[name] = h
        cost = sum(1 for _, ops in prog if len(ops) > 1)
        if best is None or cost < best[0]:
            best = (cost, prog)
    return best
