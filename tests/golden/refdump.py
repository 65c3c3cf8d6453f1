"""Reader for oracle/ref_driver.f90 dumps (stream records, little endian)."""
import numpy as np

R4_FIELDS = ["lu", "luu", "luh", "lcu", "lcv", "llu", "llv",
             "dx", "dy", "dxt", "dyt", "dxh", "dyh", "dxb", "dyb", "rlh_s", "r_diss"]
R8_FIELDS = ["ssh", "sshn", "sshp", "ubrtr", "ubrtrn", "ubrtrp", "vbrtr", "vbrtrn", "vbrtrp",
             "hhq", "hhq_p", "hhq_n", "hhu", "hhu_p", "hhu_n", "hhv", "hhv_p", "hhv_n",
             "hhh", "hhh_p", "hhh_n", "hhq_rest", "vort", "str_t", "str_s", "mu",
             "RHSx", "RHSy", "RHSx_adv", "RHSy_adv", "RHSx_dif", "RHSy_dif"]


def read_dump(path):
    """-> list of (info dict, {field: Fortran-ordered array}) per block."""
    raw = open(path, "rb").read()
    pos = 0

    def take(dt, count):
        nonlocal pos
        a = np.frombuffer(raw, dtype=dt, count=count, offset=pos)
        pos += a.nbytes
        return a

    bcount, ntr = (int(v) for v in take("<i4", 2))
    out = []
    for _ in range(bcount):
        bm, bn, nxs, nxe, nys, nye, bx1, bx2, by1, by2 = (int(v) for v in take("<i4", 10))
        shape = (bx2 - bx1 + 1, by2 - by1 + 1)
        n = shape[0] * shape[1]
        f = {}
        for name in R4_FIELDS:
            f[name] = take("<f4", n).reshape(shape, order="F").copy(order="F")
        names = list(R8_FIELDS)
        if ntr > 0:
            names += ["flux_x", "flux_y"] + [f"{p}_{t}" for t in range(1, ntr + 1) for p in ("ff1", "ff1p", "ff1n")]
        for name in names:
            f[name] = take("<f8", n).reshape(shape, order="F").copy(order="F")
        out.append((dict(bm=bm, bn=bn, nxs=nxs, nxe=nxe, nys=nys, nye=nye,
                         bx1=bx1, bx2=bx2, by1=by1, by2=by2), f))
    assert pos == len(raw), (pos, len(raw))
    return out
