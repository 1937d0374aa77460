"""Occupancy of the shared work queue of the round-5 sort that hung (block_introsort of commit
842a2c9, kBsQueue = 128 slots): four waves take ranges from one LIFO queue and push every right part,
one partition step per wave per turn, on the inputs of test_device_exact_sort_matches_std_sort.
Prints the largest number of pending ranges (never above 17, so the queue could not
overflow into its lock / counter words)."""
import sys
import numpy as np
sys.setrecursionlimit(10000)
def median_to_first(a, rf, rl):
    x, y, z = rf+1, rf+(rl-rf)//2, rl-1
    va, vb, vc = a[x], a[y], a[z]
    if va < vb: m = y if vb < vc else (z if va < vc else x)
    else: m = x if va < vc else (z if vb < vc else y)
    a[rf], a[m] = a[m], a[rf]
def partition(a, rf, rl):
    median_to_first(a, rf, rl); P = a[rf]
    i, j = rf+1, rl
    while True:
        while a[i] < P: i += 1
        j -= 1
        while P < a[j]: j -= 1
        if not i < j: return i
        a[i], a[j] = a[j], a[i]; i += 1
def run(vals, W=4, order="lifo"):
    a = list(vals); n = len(a)
    lg = n.bit_length()-1
    q = [(0, n, 2*lg)]; maxtop = 1
    waves = [None]*W   # current (rf, rl, rd) or None
    ticks = 0
    while q or any(w is not None for w in waves):
        ticks += 1
        for k in range(W):
            w = waves[k]
            if w is None:
                if q: waves[k] = q.pop(); 
                continue
            rf, rl, rd = w
            if rl - rf > 64 and rd > 0:
                rd -= 1
                cut = partition(a, rf, rl)
                q.append((cut, rl, rd)); maxtop = max(maxtop, len(q))
                waves[k] = (rf, cut, rd)
            else:
                waves[k] = None  # leaf done in one tick
    return maxtop, ticks
rng = np.random.default_rng(11)
worst = 0
for n in (700, 1024, 1800, 2048):
    for levels in (1, 3, 20, 1000):
        v = (rng.integers(0, levels, n)*0.25).tolist()
        m, t = run(v); worst = max(worst, m); print(n, levels, m)
k = 1024
killer = []
for i in range(k): killer.append((i+1) if i % 2 == 0 else (k+i+1))
killer += [2*(i+1) for i in range(k)]
print("killer", run(killer)); print("killer/3", run([x//3 for x in killer]))
