"""Per-launch HBM traffic of a kernel from rocprofv3 --pmc CSVs.

Correction (MI355X_MICROARCH.md §HBM, gfx950): FETCH_SIZE (KiB) counts
TCC_EA0_RDREQ x 64 B and reads exactly half of a wide coalesced stream's
bytes, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KiB) is exact for
wide streaming stores: write bytes = WRITE_SIZE x 1024. FETCH_SIZE and
WRITE_SIZE are collected in separate passes (TCC slot limits).

Usage: python tools/pmc_traffic.py <fetch_csv> <write_csv> [kernel_substring]
"""
import csv
import json
import sys


def per_launch(csv_path, counter, kernel_sub):
    vals = []
    with open(csv_path) as f:
        for r in csv.DictReader(f):
            if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise ValueError("no %s samples for kernel %r in %s" % (counter, kernel_sub, csv_path))
    return sum(vals) / len(vals), len(vals)


def per_call(csv_path, counter, kernel_sub, calls):
    """Sum of ``counter`` over every dispatch whose name contains ``kernel_sub``,
    divided by ``calls`` (API calls that each launch several kernels: the
    heavy-row split runs the light rows, the chunks and the combine)."""
    total, n = 0.0, 0
    with open(csv_path) as f:
        for r in csv.DictReader(f):
            if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
                total += float(r["Counter_Value"])
                n += 1
    if not n:
        raise ValueError("no %s samples for kernel %r in %s" % (counter, kernel_sub, csv_path))
    return total / calls, n


def traffic_per_call(fetch_csv, write_csv, calls, kernel_sub="gspmm"):
    fetch_kib, n1 = per_call(fetch_csv, "FETCH_SIZE", kernel_sub, calls)
    write_kib, n2 = per_call(write_csv, "WRITE_SIZE", kernel_sub, calls)
    read_b = 2.0 * fetch_kib * 1024
    write_b = write_kib * 1024
    return {"read_bytes": read_b, "write_bytes": write_b, "bytes": read_b + write_b,
            "raw_fetch_kib": fetch_kib, "raw_write_kib": write_kib, "dispatches": [n1, n2],
            "calls": calls}


def traffic(fetch_csv, write_csv, kernel_sub="gspmm_sum_kernel"):
    fetch_kib, n1 = per_launch(fetch_csv, "FETCH_SIZE", kernel_sub)
    write_kib, n2 = per_launch(write_csv, "WRITE_SIZE", kernel_sub)
    read_b = 2.0 * fetch_kib * 1024
    write_b = write_kib * 1024
    return {"read_bytes": read_b, "write_bytes": write_b, "bytes": read_b + write_b,
            "raw_fetch_kib": fetch_kib, "raw_write_kib": write_kib, "launches": [n1, n2]}


if __name__ == "__main__":
    sub = sys.argv[3] if len(sys.argv) > 3 else "gspmm_sum_kernel"
    print(json.dumps(traffic(sys.argv[1], sys.argv[2], sub), indent=1))
