#!/usr/bin/env python3
"""Writes tests/golden/lru_hash_vectors.json: the reference's own LRU test restated as data.

Source: emulator/maps_hash_lru_test.go:11-124 (TestEmulatedHashMapLRU). The Go test builds a
BPF_MAP_TYPE_LRU_HASH with KeySize 4, ValueSize 4, MaxEntries 5; keys and values are MemoryPtrs to
4-slot ValueMemories holding one IMM (makeMemPtr, :30-42), so their bytes are the little-endian u32 of
the integer (ValueMemory.ReadRange of a 4-byte run, emulator/memory.go:55-95). It updates keys 1..5
with values 11..15 (:51-71), looks up 1 then 2 (:75-83), updates 6 -> 16 (:85-89) and checks that the
UsageList is [6, 2, 1, 5, 4] (:106-123). The constants below are read off those lines; nothing of the
reference is imported or run.
"""
import json
from pathlib import Path

ops = [["update", k, 10 + k] for k in (1, 2, 3, 4, 5)] + [["lookup", 1], ["lookup", 2], ["update", 6, 16]]
out = {
    "source": "emulator/maps_hash_lru_test.go:11-124",
    "map": {"type": 9, "key_size": 4, "value_size": 4, "max_entries": 5},
    "encoding": "keys and values are little-endian u32 of the integers",
    "ops": ops,
    "expect_usage": [6, 2, 1, 5, 4],
    "expect_entries": {str(k): 10 + k for k in (1, 2, 4, 5, 6)},
}
Path(__file__).with_name("lru_hash_vectors.json").write_text(json.dumps(out, indent=1) + "\n")
print("wrote lru_hash_vectors.json")
