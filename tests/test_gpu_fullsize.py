"""C2 at the exact bench size (BASELINE.json configs[1]: 100M events, 1M keys, Zipf 1.1,
family filter, top-20 by ["-sent","-recv"]) against the oracle:
  - group count;
  - the WHOLE group table through an order-independent checksum: every group's key fields,
    sent, recv and first index fingerprinted (oracle group_csum) and summed -- the device
    table is gathered to the host and fingerprinted by the numpy twin, the oracle computes
    its own inside the all-cores restatement (or_top_tcp_mt);
  - the top-20 rows bit-exact (first, sent, recv) -- the tie order of the reference sort.
"""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, G, K = 100_000_000, 1_000_000, 20


def test_c2_full_size_table_and_topk(oracle, igx, torch):
    E, H, A = igx.engine, igx.columns, igx._abi
    bench = importlib.import_module("bench")
    cdf = E.zipf_cdf(G, 1.1)
    ev = E.gen_tcp(0xC2, 0, G, H.to_device(cdf), 0, N)
    cols = [ev[k] for k in bench.TCP_NAMES]
    tab = E.Table([16, 16, 8, 4, 16, 2, 2, 2], [A.Agg(A.AGG_SUM, 8, 9, 8, 0), A.Agg(A.AGG_SUM, 8, 9, 8, 1)],
                  G + G // 4)
    tab.update(cols, list(range(8)), N, 0, [bench.family_in_pred(A, 7)])
    fin = tab.finalize()
    top = H.host(tab.gather(tab.sort([(A.TSRC_AGG, 0, True), (A.TSRC_AGG, 1, True)], K)))
    rows = H.host(bench.table_rows(E, torch, tab, fin))
    tab.destroy()
    del ev, cols
    torch.cuda.empty_cache()
    # device packed key: saddr 0:16 daddr 16:32 mntns 32:40 pid 40:44 comm 44:60 lport 60:62
    # dport 64:66 family 68:70 (each column padded to 4 B) | sent 72 | recv 80 | first 88
    fields = np.concatenate([rows[:, 0:62], rows[:, 64:66], rows[:, 68:70]], axis=1)
    u64 = lambda o: rows[:, o:o + 8].copy().view(np.uint64).ravel()   # noqa: E731
    dev_cs = oracle.tcp_group_checksum(fields, u64(72), u64(80), u64(88))
    h = oracle.gen_tcp(0xC2, 0, G, cdf, 0, N)
    Gref, sent, recv, first, ref_cs = oracle.top_tcp_mt(h, K, checksum=True)
    assert fin["n_groups"] == Gref == rows.shape[0]
    assert dev_cs == ref_cs
    t64 = lambda o: top[:, o:o + 8].copy().view(np.uint64).ravel()    # noqa: E731
    assert np.array_equal(t64(88), first) and np.array_equal(t64(72), sent) and np.array_equal(t64(80), recv)
