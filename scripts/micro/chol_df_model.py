#!/usr/bin/env python3
"""Discrete-event model of the dataflow Cholesky (csrc/chol.h chol_solve_df)
at T = 8 tiles with six worker waves: the chain wave runs S(p+1, p),
U(p+1, p+1, p), F(p+1) per panel; worker task k goes to worker k % 6 in the
kernel's task order (panel by panel: TRSMs S(I, p), I >= p + 2, then the
updates column by column), and each wave runs its tasks in order, starting a
task when its inputs are final.  Costs are cycles per task (the measured
per-phase profiles of DESIGN.md section 3.1); prints the chain's end time,
its waits and the workers' end time for a grid of chain-factor and
worker-task costs.

Usage: chol_df_model.py [chain_factor_cycles worker_task_cycles]
"""
import sys

T, NWK = 8, 6
CS, CU = 1890, 1000   # chain TRSM / chain update (fused into the factor)
WB = 400              # a worker TRSM's rhs update B(I, p)


def deps(t):
    if t[0] == "F":
        p = t[1]
        return [("U", p, p, p - 1)] if p > 0 else []
    if t[0] == "S":
        i, p = t[1], t[2]
        return [("F", p)] + ([("U", i, p, p - 1)] if p > 0 else [])
    i, j, p = t[1], t[2], t[3]
    return [("S", i, p), ("S", j, p)] + ([("U", i, j, p - 1)] if p > 0 else [])


def worker_tasks():
    order = []
    for p in range(T - 1):
        order += [("S", i, p) for i in range(p + 2, T)]
        for j in range(p + 1, T):
            order += [("U", i, j, p) for i in range(p + 2 if j == p + 1 else j, T)]
    return order


def simulate(cf, wt):
    chain = []
    for p in range(-1, T - 1):
        if p >= 0:
            chain += [("S", p + 1, p), ("U", p + 1, p + 1, p)]
        chain.append(("F", p + 1))
    waves = [[] for _ in range(NWK)]
    for k, t in enumerate(worker_tasks()):
        waves[k % NWK].append(t)
    seqs = [chain] + waves
    cost = [{"F": cf, "S": CS, "U": CU}] + [{"S": wt + WB, "U": wt}] * NWK
    done, pos = {}, [0] * len(seqs)
    now, wait = [0.0] * len(seqs), [0.0] * len(seqs)
    progress = True
    while progress:
        progress = False
        for i, seq in enumerate(seqs):
            while pos[i] < len(seq):
                t = seq[pos[i]]
                if not all(d in done for d in deps(t)):
                    break
                start = max([now[i]] + [done[d] for d in deps(t)])
                wait[i] += start - now[i]
                now[i] = start + cost[i][t[0]]
                done[t] = now[i]
                pos[i] += 1
                progress = True
    assert all(pos[i] == len(s) for i, s in enumerate(seqs)), "deadlock"
    return now[0], wait[0], max(now[1:])


def main():
    if len(sys.argv) == 3:
        grid = [(float(sys.argv[1]), float(sys.argv[2]))]
    else:
        grid = [(cf, wt) for cf in (6800, 5500, 4500) for wt in (3600, 3200, 2800, 2400)]
    for cf, wt in grid:
        c, w, e = simulate(cf, wt)
        print(f"factor {cf:6.0f}  worker task {wt:6.0f}:  chain {c:7.0f}  "
              f"chain waits {w:6.0f}  workers end {e:7.0f}")


if __name__ == "__main__":
    main()
