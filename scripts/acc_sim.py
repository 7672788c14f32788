#!/usr/bin/env python3
"""Why C3's map adds reach HBM: replay the per-wave LDS accumulator policy of
xe_interp.h wave_atomic_add_field on C3's packet stream, CPU only.

Each wave walks 64-packet chunks w, w + nwaves, ... (parallel_packets); per chunk the 64 lanes make one
add each on a hit (90 % of C3's packets), in lane order. The table: XE_ACC direct-mapped entries by
acc_slot(field address), claimed when free, taken over when misses wear the owner's score down (the old
sum flushed to HBM), flushed once per owned entry when the wave retires. An add that misses goes to HBM
as one atomic; the memory side counts one request per 64-B line per wave-instruction, so the misses of
one chunk are grouped by line. Flow -> hash slot is a fixed random map (the device table's slots are a
hash of the key), value_size 16 -> four values per line.

  python scripts/acc_sim.py [waves=256] [acc sizes...]    -> JSON lines (profiles/r4/c3_acc_sim.json)
"""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from gobpfld_amd import workloads as W  # noqa: E402

NWAVES_GRID = 4096          # 1024 blocks x 4 waves (16 waves per CU x 256 CUs)
CHUNKS_PER_WAVE = 64        # 16,777,216 packets / 64 / 4096
CAP = 1 << 21               # C3's HASH table: pow2 >= 2 x MaxEntries (1M)


def stream(wave: int):
    """flow id per packet (-1: a miss, no add) of wave `wave`'s chunks, in order"""
    chunks = wave + NWAVES_GRID * np.arange(CHUNKS_PER_WAVE, dtype=np.uint64)
    idx = (chunks[:, None] * np.uint64(64) + np.arange(64, dtype=np.uint64)[None, :]).reshape(-1)
    r0 = W.rng_stream(3, idx, 0)
    u = (r0 >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    hit = (W.rng_stream(3, idx, 2) % np.uint64(10)) != 0
    fid = W.zipf_ranks(u, W.C3_FLOWS).astype(np.int64)
    return np.where(hit, fid, -1).reshape(CHUNKS_PER_WAVE, 64)


def acc_slot(addr: int, acc: int) -> int:
    """xe_interp.h acc_slot: the top log2(XE_ACC) bits of a multiplicative hash (XE_ACC_BITS)"""
    bits = acc.bit_length() - 1
    return ((((addr >> 2) * 0x9E3779B97F4A7C15) & ((1 << 64) - 1)) >> (64 - bits)) & (acc - 1)


def simulate(waves: int, acc: int, slot_of: np.ndarray) -> dict:
    adds = lds = hbm_adds = hbm_req = flush_req = 0
    for w in range(waves):
        tag = [0] * acc
        score = [0] * acc
        summ = [0] * acc
        for chunk in stream(w):
            miss_lines = set()
            for f in chunk:
                if f < 0:
                    continue
                adds += 1
                addr = 0x100000000 + int(slot_of[f]) * 16 + 8   # the hits counter of the flow's value
                k = acc_slot(addr, acc)
                t = tag[k]
                if t == 0:
                    tag[k] = addr
                    score[k] = 1
                elif t != addr:
                    score[k] -= 1
                    if score[k] + 1 <= 1:   # xe_lds_add32 returns the old value
                        if summ[k]:
                            flush_req += 1
                        tag[k], summ[k], score[k] = addr, 0, 2
                if tag[k] == addr:
                    summ[k] += 1
                    if t == addr:
                        score[k] += 1
                    lds += 1
                else:
                    hbm_adds += 1
                    miss_lines.add(addr >> 6)
            hbm_req += len(miss_lines)
        flush_req += sum(1 for k in range(acc) if tag[k] and summ[k])
    pk = waves * CHUNKS_PER_WAVE * 64
    return {"acc_entries": acc, "packets": pk, "adds_per_pkt": adds / pk, "lds_hit_rate": lds / adds,
            "hbm_adds_per_pkt": hbm_adds / pk, "atomic_requests_per_pkt": (hbm_req + flush_req) / pk,
            "flush_requests_per_pkt": flush_req / pk}


def top_share(k: int) -> float:
    w = 1.0 / np.power(np.arange(1, W.C3_FLOWS + 1, dtype=np.float64), 1.1)
    return float(w[:k].sum() / w.sum())


if __name__ == "__main__":
    waves = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    sizes = [int(x) for x in sys.argv[2:]] or [64, 128, 256, 512]
    slot_of = np.random.default_rng(7).choice(CAP, size=W.C3_FLOWS, replace=False)
    for acc in sizes:
        r = simulate(waves, acc, slot_of)
        r["zipf_top_k_share_of_hits"] = top_share(acc)
        print(json.dumps(r), flush=True)
