"""Host simulation of the Server's encoder waste under slot-refill policies:
4096 slots in 128-row tiles, 128-frame chunks, dev-clean lengths, saturated queue.  A round
computes, per frame of the chunk, every row of every active tile: "prefix" = the tick kernel's
structure today (tiles up to the last one still running), "tile list" = a kernel that skips any
tile whose rows are done.  Policies: fcfs (free slots take the oldest samples), group (a tile is
refilled when empty, with samples of the oldest one's chunk count), near (a tile is refilled when
empty, with the oldest sample and the pending ones closest to its length).  Prints useful /
computed row-frames and samples finished per round."""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))), 'rnnt-inference_amd'))
from rnnt_amd import synthetic
L, S, TILE = 128, 4096, 128
lens_pool = synthetic.devclean_lengths(2513, seed=1)
rng = np.random.default_rng(0)
def run(policy, rounds=400, window=2048, tile_list=False):
    nt = S // TILE
    rem = np.zeros(S, np.int64)           # frames left per slot (0 = free)
    pending = list(rng.choice(lens_pool, 20000))
    useful = computed = 0; done = 0
    for r in range(rounds):
        # refill
        if policy == 'fcfs':
            free = np.nonzero(rem == 0)[0]
            k = min(len(free), len(pending))
            rem[free[:k]] = pending[:k]; del pending[:k]
        else:
            for t in range(nt):
                sl = slice(t * TILE, (t + 1) * TILE)
                if (rem[sl] == 0).all() and pending:
                    if policy == 'tile':
                        take = pending[:TILE]; del pending[:TILE]
                    elif policy == 'near':  # the oldest sample and the pending ones closest to its length
                        win = pending[:window]
                        x0 = win[0]
                        idx = sorted(range(len(win)), key=lambda i: (abs(win[i] - x0), i))[:TILE]
                        take = [win[i] for i in idx]
                        for i in sorted(idx, reverse=True): del pending[i]
                    else:  # tile + group by chunk count of the oldest sample
                        win = pending[:window]
                        c0 = -(-win[0] // L)
                        idx = [i for i, x in enumerate(win) if -(-x // L) == c0][:TILE]
                        if len(idx) < TILE:  # fill with the closest chunk counts
                            rest = sorted((i for i in range(len(win)) if i not in set(idx)), key=lambda i: abs(-(-win[i] // L) - c0))
                            idx += rest[:TILE - len(idx)]
                        take = [win[i] for i in idx]
                        for i in sorted(idx, reverse=True): del pending[i]
                    rem[t * TILE: t * TILE + len(take)] = take
        busy = rem > 0
        ch = np.where(busy, np.minimum(rem, L), 0)
        tmax = ch.reshape(nt, TILE).max(1)
        # active prefix per frame t: tiles up to the last with tmax > t
        if tile_list:
            computed += int(tmax.sum()) * TILE
        else:
          for t in range(int(tmax.max()) if busy.any() else 0):
            act = np.nonzero(tmax > t)[0]
            computed += (act[-1] + 1) * TILE
        useful += ch.sum()
        rem = rem - ch
        done += int((busy & (rem == 0)).sum())
        pending += list(rng.choice(lens_pool, int((busy & (rem == 0)).sum()) + 0))  # keep saturated
    return useful / computed, done / rounds
for tl in (False, True):
  for p in ('fcfs', 'group', 'near'):
    eff, thr = run(p, tile_list=tl)
    print('tile list' if tl else 'prefix', p, 'useful/computed %.3f' % eff, 'samples per round %.1f' % thr)
