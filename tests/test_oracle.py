"""The oracle is pinned against the golden vectors produced by the reference's
own arithmetic (torch.sparse.mm on the reference's COO; tests/golden/make_golden.py)."""
import numpy as np

from oracle import oracle as O


def _np(a):
    return np.asarray(a)


def test_spmm_copy_and_mul_bit_exact(golden):
    for name in ("spec10", "cora", "multi", "zerodeg"):
        c = golden(name)
        n = int(c["n"])
        out = O.spmm_coo(n, c["dst"], c["src"], c["h"])
        assert np.array_equal(out, c["copy_out"]), name
        if "mul_out" in c:
            out = O.spmm_coo(n, c["dst"], c["src"], c["h"], c["w"])
            assert np.array_equal(out, c["mul_out"]), name


def test_backward_is_transposed_chain(golden):
    """dH = A^T dC: the same fma chain over out-edges in edge-id order."""
    for name in ("spec10", "cora", "multi"):
        c = golden(name)
        n = int(c["n"])
        gh = O.spmm_coo(n, c["src"], c["dst"], c["g"])
        assert np.array_equal(gh, c["copy_grad_h"]), name
        if "mul_grad_h" in c:
            gh = O.spmm_coo(n, c["src"], c["dst"], c["g"], c["w"])
            assert np.array_equal(gh, c["mul_grad_h"]), name
            gw = O.sddmm_dot(c["dst"], c["src"], c["g"], c["h"])
            np.testing.assert_allclose(gw, c["mul_grad_w"], rtol=1e-5, atol=1e-5)


def test_csr_form_and_openmp_equal_coo(golden):
    c = golden("cora")
    n = int(c["n"])
    indptr, indices, pos = O.coo_to_csr(n, c["dst"], c["src"])
    assert indptr[-1] == len(c["src"])
    assert np.all(np.diff(pos[indptr[1]:indptr[2]]) > 0)
    for threads in (1, 4):
        out = O.spmm_csr(indptr, indices, pos, c["h"], num_threads=threads)
        assert np.array_equal(out, c["copy_out"])


def test_python_restatement(golden):
    c = golden("spec10")
    out = O.spmm_coo_py(int(c["n"]), c["dst"], c["src"], c["h"], c["w"])
    assert np.array_equal(out, c["mul_out"])


def test_max_mean_mailbox(golden):
    c = golden("multi")
    n = int(c["n"])
    msgs = c["h"][c["src"]]
    assert np.array_equal(O.max_mailbox(n, c["dst"], msgs), c["max_out"])
    np.testing.assert_allclose(O.mean_mailbox(n, c["dst"], msgs), c["mean_out"],
                               rtol=1e-6, atol=1e-6)
    z = golden("zerodeg")
    assert np.array_equal(O.max_mailbox(int(z["n"]), z["dst"], z["h"][z["src"]]), z["max_out"])


def test_snr_rectangular(golden):
    c, s = golden("cora"), golden("snr")
    u, v = c["src"][s["sel"]], c["dst"][s["sel"]]
    rows = np.searchsorted(s["recv"], v)
    out = O.spmm_coo(len(s["recv"]), rows, u, c["h"])
    assert np.array_equal(out, s["out"])


def test_feat3d(golden):
    c = golden("feat3d")
    n = int(c["n"])
    out = O.spmm_coo(n, c["dst"], c["src"], c["h"].reshape(n, 25)).reshape(n, 5, 5)
    assert np.array_equal(out, c["copy_out"])


def _reddit_rows_inputs(golden):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import portable as P
    c = golden("reddit_rows")
    src, dst, H, W, G = P.reddit_rows()
    for k, a in (("src", src), ("dst", dst), ("h", H), ("w", W), ("g", G)):
        assert P.digest(a) == str(c["sha_" + k]), "portable generator drifted: " + k
    return c, P, src, dst, H, W, G


def test_reddit_rows_fixture(golden):
    """Reddit row lengths (rows of 13k-54k in-edges, thousands of parallel
    duplicates, 1.5M edges, F = 128): the oracle's chain equals
    torch.sparse.mm on the reference's uncoalesced COO bit for bit, for
    copy_u and u_mul_e, forward and dH, over the whole output (digest) and a
    row sample (stored rows). The OpenMP CSR form (the multi-core CPU
    baseline) gives the same bits."""
    c, P, src, dst, H, W, G = _reddit_rows_inputs(golden)
    n = int(c["n"])
    assert int(c["max_in_degree"]) >= 20000
    rows = c["rows"]
    outs = {"copy_out": O.spmm_coo(n, dst, src, H),
            "mul_out": O.spmm_coo(n, dst, src, H, W),
            "copy_grad_h": O.spmm_coo(n, src, dst, G),
            "mul_grad_h": O.spmm_coo(n, src, dst, G, W)}
    for k, out in outs.items():
        assert np.array_equal(out[rows], c[k + "_rows"]), k
        assert P.digest(out) == str(c["sha_" + k]), k
    ip, ix, pos = O.coo_to_csr(n, dst, src)
    assert P.digest(O.spmm_csr(ip, ix, pos, H, num_threads=8)) == str(c["sha_copy_out"])
    assert P.digest(O.spmm_csr(ip, ix, pos, H, W, num_threads=8)) == str(c["sha_mul_out"])
