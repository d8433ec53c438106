"""Oracle composition of the fused key-switch forms (test helper; oracle/oracle.c restates the
reference functions): relinearize + rescale = moddown_from_NTT over the special basis {q_last} u P
of the P-scaled (c0, c1) + key_switch_inner_prod(modup(c2)) (src/rns_bconv.cu:530-843,
src/eval_key_switch.cu:26-85)."""
import numpy as np

import oracle_lib as O


def relinearize_rescale(ctx, chain, ct, keys):
    """ct: [3][L][n] (numpy u64) at `chain`; keys: dnum numpy digits [2][size_QP][n].
    Returns [2][L-1][n]."""
    ql, p = ctx.ql(chain), ctx.moduli[ctx.size_Q:]
    L, n = len(ql), ctx.n
    beta = -(-L // ctx.size_P)
    qlp = list(ql) + list(p)
    tmu = np.zeros(beta * len(qlp) * n, dtype=np.uint64)
    O.lib().or_modup(O.P(ct[2 * L * n:3 * L * n].copy()), O.P(tmu), n, O.P(O.arr(ql)), L, O.P(O.arr(p)), len(p))
    cx = np.zeros(2 * len(qlp) * n, dtype=np.uint64)
    okeys = (O.u64p * len(keys))(*[O.P(k) for k in keys])
    O.lib().or_keyswitch_inner_prod(O.P(tmu), okeys, O.P(cx), n, L, ctx.size_Q, ctx.size_P, beta,
                                    O.P(O.arr(ctx.moduli)))
    P = 1
    for v in p:
        P *= int(v)
    pmod = O.arr([P % int(q) for q in ql])
    want = []
    for t in range(2):
        c = cx[t * len(qlp) * n:(t + 1) * len(qlp) * n].copy()
        scaled = np.zeros(L * n, dtype=np.uint64)
        O.lib().or_poly_mul_scalar(O.P(ct[t * L * n:(t + 1) * L * n].copy()), O.P(pmod), O.P(scaled), n, L,
                                   O.P(O.arr(ql)))
        O.lib().or_poly_add(O.P(c[:L * n].copy()), O.P(scaled), O.P(c[:L * n]), n, L, O.P(O.arr(ql)))
        w = np.zeros((L - 1) * n, dtype=np.uint64)
        O.lib().or_moddown_from_ntt(O.P(c), O.P(w), n, O.P(O.arr(ql[:-1])), L - 1, O.P(O.arr([ql[-1]] + list(p))),
                                    len(p) + 1)
        want.append(w)
    return np.concatenate(want)
