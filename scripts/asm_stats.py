"""Instruction histogram of one kernel in a hipcc -S output: python scripts/asm_stats.py file.s substr"""
import collections
import sys

s = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(s) if sys.argv[2] in l and l.endswith(":") or (sys.argv[2] in l and ": ;" in l))
c = collections.Counter()
loops = 0
for l in s[start + 1:]:
    l = l.strip()
    if l.startswith(".Lfunc_end"):
        break
    if not l or l.startswith(";") or l.startswith("."):
        continue
    c[l.split()[0]] += 1
ops = sys.argv[3:] or ["v_accvgpr_read_b32", "v_accvgpr_write_b32", "v_accvgpr_mov_b32", "v_mfma_f32_16x16x32_bf16",
                       "s_waitcnt", "scratch_store_dword", "scratch_load_dword", "v_writelane_b32", "v_readlane_b32",
                       "s_barrier", "buffer_load_dword", "ds_read_b64_tr_b16", "ds_read_b128", "ds_write_b64"]
for op in ops:
    print(op, c[op])
print("total", sum(c.values()))
