"""Static check of counted seam waits against the emitted listing: the split training
forward (mlp_x3.h, TrainVm; kernel mlp_x3_kernel<false, true, OpBf16>) and the split
backward-data chain (train_bwd_x3.hip, kVm; kernel train_bwd_x3_kernel).

Walking the tile loop's straight-line body, at every seam (an `s_waitcnt vmcnt(N)`
followed by `s_barrier`) the chunk the barrier publishes was staged by the stage group
after the barrier `--back` seams earlier (the tile top counts as one: both kernels run a
4-slot ring, chunk j staged at seam j - 3 and needed at seam j - 1).  A stage group is the
first `--pieces` LDS-DMA pieces issued after that barrier (other LDS-DMA issued right after
them -- the backward's mask-word piece -- is younger, as the kernels' tables count it).  The
wait is sound when N <= the vector-memory operations issued after the group's last piece;
a table that counted more operations than the compiler emitted fails here.

    python tools/check_train_seams.py LISTING.s [--kernel REGEX] [--pieces N] [--back K]
"""
import argparse
import re
import sys

VMEM = re.compile(r"^\s*(global_|buffer_|scratch_|flat_)")
KERNELS = {
    "mlp_bf16x3": r"_ZN4nerf12_GLOBAL__N_113mlp_x3_kernelILb0ELb1E\S*",
    "train_bwd_x3": r"_ZN4nerf12_GLOBAL__N_119train_bwd_x3_kernel\S*",
}


def check(path, kernel, pieces=None, back=2, verbose=True):
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(rf"^{kernel}:", l)]
    if not starts:
        raise SystemExit(f"{path}: no kernel matching {kernel}")
    start = starts[0]
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

    def group_end(bi):
        """Index of the last piece of the stage group after barrier bi: the first `pieces`
        LDS-DMA ops (or, without `pieces`, the first contiguous run of them)."""
        j, last, n = bi + 1, None, 0
        while j < len(ev) and ev[j][0] != "barrier":
            if ev[j][0] == "vm" and ev[j][1]:
                last, n = j, n + 1
                if pieces is not None and n == pieces:
                    return last
            elif ev[j][0] == "vm" and last is not None:
                break
            j += 1
        return last if pieces is None else None

    bad, checked = 0, 0
    for k in range(back, len(seams)):
        bi, n = seams[k]
        if n is None:
            continue
        g_end = group_end(seams[k - back][0])
        if g_end is None:
            continue
        younger = sum(1 for e in ev[g_end + 1:bi] if e[0] == "vm")
        checked += 1
        if n > younger:
            bad += 1
            print(f"seam {k}: vmcnt({n}) but only {younger} vector-memory ops after the chunk it publishes")
    if verbose:
        print(f"{path} [{kernel}]: {checked} counted seams checked, {bad} unsound; {len(seams)} barriers")
    return checked, bad


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("listing")
    ap.add_argument("--kernel", default=None, help="symbol regex, or one of " + ", ".join(KERNELS))
    ap.add_argument("--pieces", type=int, default=None, help="LDS-DMA pieces per stage group per wave")
    ap.add_argument("--back", type=int, default=2, help="seams between a chunk's stage and its publication")
    ap.add_argument("--min-checked", type=int, default=1, help="fail unless at least this many seams were checked")
    a = ap.parse_args(argv)
    kernel = KERNELS.get(a.kernel, a.kernel) if a.kernel else KERNELS["mlp_bf16x3"]
    checked, bad = check(a.listing, kernel, a.pieces, a.back)
    if checked < a.min_checked:
        print(f"only {checked} seams checked (< {a.min_checked}): the listing no longer matches the checker")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
