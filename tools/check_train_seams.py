"""Static check of the split training forward's counted seam waits (mlp_x3.h, TrainVm) on
the emitted listing: walking the tile loop's straight-line body, at every seam (an
`s_waitcnt vmcnt(N)` followed by `s_barrier`) the chunk the barrier publishes was staged by
the LDS-DMA group after the barrier two seams back (the tile top counts as one); the wait
is sound when N <= the vector-memory operations issued after that group's last piece.

    python tools/check_train_seams.py nerf-dbr_amd/csrc/build/asm/mlp_bf16x3.s
"""
import re
import sys

VMEM = re.compile(r"^\s*(global_|buffer_|scratch_|flat_)")


def main(path):
    lines = open(path).read().split("\n")
    start = [i for i, l in enumerate(lines) if re.match(r"^_ZN4nerf12_GLOBAL__N_113mlp_x3_kernelILb0ELb1E\S*:", l)][0]
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = [l.split(";")[0].strip() for l in lines[start:end]]
    body = [l for l in body if l and not l.startswith(".")]
    # events in order: ('vm', is_dma), ('wait', n), ('barrier',)
    ev = []
    for l in body:
        if VMEM.match(l):
            ev.append(("vm", "global_load_lds" in l))
        m = re.match(r"s_waitcnt\s+.*vmcnt\((\d+)\)", l)
        if m:
            ev.append(("wait", int(m.group(1))))
        if l.startswith("s_barrier"):
            ev.append(("barrier",))
    # seam = barrier preceded (directly, ignoring non-vm events) by a wait
    seams = []       # (index of barrier in ev, wait count)
    last_wait = None
    for i, e in enumerate(ev):
        if e[0] == "wait":
            last_wait = e[1]
        elif e[0] == "vm":
            last_wait = None
        elif e[0] == "barrier":
            seams.append((i, last_wait))
            last_wait = None
    # the DMA group after each barrier: index of its last piece
    def group_end(bi):
        j, last = bi + 1, None
        while j < len(ev) and ev[j][0] != "barrier":
            if ev[j][0] == "vm" and ev[j][1]:
                last = j
            elif ev[j][0] == "vm" and last is not None:
                break
            j += 1
        return last
    bad, checked = 0, 0
    for k in range(2, len(seams)):
        bi, n = seams[k]
        if n is None:
            continue
        g_end = group_end(seams[k - 2][0])
        if g_end is None:
            continue
        younger = sum(1 for e in ev[g_end + 1:bi] if e[0] == "vm")
        checked += 1
        if n > younger:
            bad += 1
            print(f"seam {k}: vmcnt({n}) but only {younger} vector-memory ops after the chunk it publishes")
    print(f"{path}: {checked} counted seams checked, {bad} unsound; {len(seams)} barriers")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
