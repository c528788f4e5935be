#!/usr/bin/env python3
"""Slot simulation of the closed-loop row wavefront: 1,024 wave
slots, one block step per time unit, block bx of row r after row r-1 finished
bx+1; compares ticket orders for 8 1080p YUV420 frames."""
import heapq, numpy as np
def sim(order, slots, rows):
    # rows: list of (plane, by, bw); dependency on (plane, by-1)
    # finish time of block bx of row: f[row][bx]
    done = {}   # (plane,by) -> array of finish times
    free = [0.0]*slots
    heapq.heapify(free)
    end = 0
    for (p, by, bw) in order:
        t0 = heapq.heappop(free)   # slot available time (tickets in order)
        f = np.zeros(bw)
        prev = done.get((p, by-1))
        t = t0
        for bx in range(bw):
            if prev is not None:
                need = min(bx+1, bw-1)   # blocks <= bx+1 done
                t = max(t, prev[need])
            t += 1.0
            f[bx] = t
        done[(p, by)] = f
        heapq.heappush(free, t)
        end = max(end, t)
    return end
F = 8
rows = []
for fr in range(F):
    for pi, (bh, bw) in enumerate([(135, 240), (67, 120), (67, 120)]):
        for by in range(bh):
            rows.append((fr*3+pi, by, bw))
plane_major = rows
by_major = sorted(rows, key=lambda r: (r[1], r[0]))
by2 = sorted(rows, key=lambda r: (2*r[1] , -r[2], r[0]))
for name, o in [("plane-major", plane_major), ("by-major", by_major), ("by2", by2)]:
    for slots in (1024, 2048):
        print(name, slots, sim(o, slots, rows))
print("work lower bound", sum(r[2] for r in rows)/1024)
