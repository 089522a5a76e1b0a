"""LDS bytes per candidate for the rollout kernel (mirror of make_layout in
csrc/mgs_capi.hip) -- a what-if tool for layout changes.  Usage:
  python tools/lds_budget.py [ncon_max] [nefc_max] [gstride_extra]"""
import sys


def layout(nq=22, nv=20, nb=18, ng=16, nu=1, nj=10, nmocap=1, nc=16, ne=None, gpad=0, K_MAXPOLY=40, BLK=16):
    if ne is None:
        ne = 4 * nc + 21
    gs = nv + gpad
    L = dict(qpos=nq, qvel=nv, qacc_ws=nv, ctrl=nu, mocap_pos=3 * nmocap + 3, mocap_quat=4 * nmocap + 4, time=1,
             xpos=3 * nb, xquat=4 * nb, xmat=9 * nb, subtree_com=3 * nb, cinert=10 * nb, cdof=6 * nv,
             M=nv * nv, Dv=nv, Dinv=nv, sD=nv, isD=nv, tmp=nv, tmp2=nv, qfrc_smooth=nv, qacc_smooth=nv,
             qfrc_constraint=nv, act_force=nu, act_moment=nu * nv, act_length=nu, act_vel=nu,
             con_pos=3 * nc, con_frame=9 * nc, con_dist=nc, con_mu=5 * nc, con_blk=BLK * nc, efc_R=ne, efc_b=ne)
    kin = 6 * K_MAXPOLY * 3 + K_MAXPOLY + 3 * ng + 9 * ng + 3 * nb + 3 * nj + 3 * nj + nb + 4 * nb
    dyn = max(10 * nb, 6 * nb * 3 + 6 * nv + 3 * nv)
    scratch = max(2 * ne, nv)
    xreg = max(3 * ne, nv * nv - scratch)
    con = ne * gs + ne + xreg + scratch + 5 * ne + 4 * nv
    U = max(kin, dyn, con, nv * nv)
    ints = (16 + 3 * nc + 4 * ne + 1) // 2
    tot = sum(L.values()) + U + ints
    return tot * 8, dict(persistent=sum(L.values()) * 8, U=U * 8, U_kin=kin * 8, U_dyn=dyn * 8, U_con=con * 8,
                         ints=ints * 8)


if __name__ == "__main__":
    nc = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    ne = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    gp = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    b, parts = layout(nc=nc, ne=ne, gpad=gp)
    print(f"{b} bytes ({b / 1024:.2f} KiB), {163840 // b} candidates per CU; {parts}")
