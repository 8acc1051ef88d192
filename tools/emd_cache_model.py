#!/usr/bin/env python3
"""Numpy model of the EMD auction's cache proofs (the analysis behind the
seed's reserve and nearest-64 cache).

Runs the auction semantics of emd_cuda.cu (as oracle/pcm_oracle.c restates
them) and, beside it, the build's per-point caches: a cache set with a value
bound, the proof `second best > bound`, and the rebuild on a miss.  Policies:
'lane' = every lane top-2 above the max of the lanes' third keys (scan_seed /
select_cache), 'top' = the exact top-L; tier2 = a reserve of every object
within a radius (FACT x the cache bound's d, shrunk until tier2 fit).  Prints
bids, misses, reserve rescues and the share of element-iterations with a full
scan.  Usage: FACT=4 python tools/emd_cache_model.py c3 [B]  (config 3), or
... tr [B] [iters] with /tmp/pred.npz holding {'pred', 'gt'} clouds.
Approximate (float64 values, no fp32 scan keys): for policy comparison only.
"""
import numpy as np, sys, time, os
FACT = float(os.environ.get('FACT', '2.5'))

def values(P, Q, J, price):
    d = ((Q[None, :, :] - P[J][:, None, :]) ** 2).sum(-1).astype(np.float32)
    s = np.sqrt(d)
    return ((3.0 - s.astype(np.float64)) - price[None, :].astype(np.float64)).astype(np.float32)

def select(v, policy, L):
    """v: [m, n] keys (larger better). returns (mask of cached [m,n], bound [m])"""
    m, n = v.shape
    if policy == 'lane':
        lanes = v.reshape(m, n // 64, 64)  # object k -> lane k % 64
        srt = -np.sort(-lanes, axis=1)
        K3 = srt[:, 2, :].max(1)
        top2 = srt[:, 1, :]  # lane 2nd best
        cand = v > K3[:, None]
        # entries above K3 are necessarily lane top-2 (3rd <= K3)
        cnt = cand.sum(1)
        bound = K3.copy()
        for i in np.nonzero(cnt > L)[0]:
            o = -np.sort(-v[i]); bound[i] = o[L]  # approx of bisection: exact L-th
            cand[i] = v[i] > bound[i]
        return cand, bound
    else:  # exact top-L
        o = -np.sort(-v, axis=1)
        bound = o[:, L]
        return v > bound[:, None], bound

def run(P1, P2, eps, iters, policy, L, tier2=0):
    B, n, _ = P1.shape
    stats = dict(bids=0, miss=0, rescue=0, iters_with_miss=0, elem_iters=0, maxmiss=[])
    for b in range(B):
        P, Q = P1[b], P2[b]
        price = np.zeros(n, np.float32)
        ass = -np.ones(n, np.int64); inv = -np.ones(n, np.int64)
        allJ = np.arange(n)
        v0 = values(P, Q, allJ, price)
        cmask, cT = select(v0, policy, L)
        if tier2:
            s = 3.0 - v0.astype(np.float64)  # price 0
            sK = 3.0 - cT.astype(np.float64)
            th = sK * np.sqrt(FACT)
            for _ in range(8):
                cnt = (s < th[:, None]).sum(1)
                over = cnt > tier2
                if not over.any(): break
                th = np.where(over, np.maximum(sK, th * np.sqrt(0.8)), th)
            t2mask = s < th[:, None]
            t2T = (3.0 - th).astype(np.float32)
            t2ok = (t2mask.sum(1) <= tier2)
            print('reserve sizes', np.percentile(t2mask.sum(1), [5, 50, 95]), 'unavailable', (~t2ok).sum())
        for it in range(iters):
            last = it == iters - 1
            U = np.nonzero(ass == -1)[0]
            if len(U) == 0:
                break
            v = values(P, Q, U, price)
            o = np.argsort(-v, axis=1, kind='stable')
            best_i = o[:, 0]
            best = v[np.arange(len(U)), best_i]
            better = v[np.arange(len(U)), o[:, 1]]
            if it > 0:
                # cache proof
                cv = np.where(cmask[U], v, -np.inf)
                c2 = -np.sort(-cv, axis=1)[:, 1]
                ok = c2 > cT[U]
                miss = np.nonzero(~ok)[0]
                stats['bids'] += len(U)
                nm = 0
                if len(miss):
                    J = U[miss]
                    if tier2:
                        tv = np.where(t2mask[J], v[miss], -np.inf)
                        t2 = -np.sort(-tv, axis=1)[:, 1]
                        resc = (t2 > t2T[J]) & t2ok[J]
                        stats['rescue'] += int(resc.sum())
                        # rebuild tier-1 from tier-2 at current prices
                        for ii in np.nonzero(resc)[0]:
                            j = J[ii]; row = tv[ii]
                            srt = -np.sort(-row)
                            thr = srt[L] if L < tier2 else -np.inf
                            cmask[j] = row > thr
                            cT[j] = max(t2T[j], thr)
                        fm = miss[~resc]
                        t2ok[U[fm]] = False
                    else:
                        fm = miss
                    nm = len(fm)
                    if nm:
                        m2, T2 = select(v[fm], policy, L)
                        cmask[U[fm]] = m2; cT[U[fm]] = T2
                stats['miss'] += nm
                stats['elem_iters'] += 1
                stats['iters_with_miss'] += nm > 0
                stats['maxmiss'].append(nm)
            inc = (best - better + np.float32(eps)).astype(np.float32)
            maxinc = {}
            for u in range(len(U)):
                k = best_i[u]
                if k not in maxinc or inc[u] > maxinc[k]: maxinc[k] = inc[u]
            claimed = {}
            for u in range(len(U)):
                k = best_i[u]; mi = float(maxinc[k]); bi = float(inc[u])
                if bi - 1e-6 <= mi <= bi + 1e-6 and k not in claimed: claimed[k] = u
            for u in range(len(U)):
                j = U[u]; k = best_i[u]
                if last: ass[j] = k
                elif claimed.get(k) == u:
                    old = inv[k]
                    if old != -1: ass[old] = -1
                    inv[k] = j; ass[j] = k; price[k] += inc[u]
    mm = np.array(stats['maxmiss'])
    return dict(bids=stats['bids'], miss=stats['miss'], rescue=stats['rescue'],
                frac_iters_miss=stats['iters_with_miss'] / max(1, stats['elem_iters']),
                mean_miss=mm.mean(), p90=np.percentile(mm, 90) if len(mm) else 0)

if __name__ == '__main__':
    which = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    if which == 'c3':
        g = np.random.default_rng(0)
        P1 = g.random((B, 1024, 3), dtype=np.float32); P2 = g.random((B, 1024, 3), dtype=np.float32)
        eps, iters = 0.005, 50
    else:
        d = np.load('/tmp/pred.npz'); P1 = d['pred'][:B]; P2 = d['gt'][:B]
        eps, iters = 0.05, int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    for pol, L, t2 in [('top', 64, 128), ('top', 64, 192), ('top', 64, 256)]:
        t = time.time()
        r = run(P1, P2, eps, iters, pol, L, t2)
        print(which, pol, L, 'tier2', t2, r, f'{time.time()-t:.1f}s', flush=True)
