"""The C-ABI library (CPU-side checks, no compute): it builds for gfx950, loads, exports every
symbol include/hgsim.h declares, and the ctypes struct layouts match the C header."""
import ctypes
import os
import re
import subprocess

import pytest

from humanoid import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "hgsim.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(hg_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_lists_exports():
    assert header_functions() == sorted(N.EXPORTS)


def test_library_exports_all_symbols():
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libhgsim.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in N.EXPORTS if s not in syms]
    assert not missing, missing


def test_library_loads_without_gpu():
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libhgsim.so not built")
    L = N.load_library()
    assert b"gfx950" in L.hg_version()
    cfg = N.HgCfg()
    assert L.hg_arena_bytes(ctypes.byref(cfg)) == 0          # num_envs = 0 -> invalid
    cfg.num_envs, cfg.frame_stack, cfg.c_frame_stack = 4096, 15, 3
    nbytes = L.hg_arena_bytes(ctypes.byref(cfg))
    # SoA state + the observation history windows (14 + 26 frames of 47, 2 + 26 frames of 73 per env)
    assert 4096 * (40 * 47 + 28 * 73) * 4 < nbytes < 128 << 20
    out = ctypes.c_void_p()
    rc = L.hg_create(ctypes.byref(cfg), None, None, 0, ctypes.byref(out))
    assert rc != 0 and b"null" in L.hg_last_error(None)


def test_struct_layouts_match_header(tmp_path):
    c = tmp_path / "sz.c"
    c.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "hgsim.h"\nint main(){printf("%zu %zu %zu %zu %zu",'
                 'sizeof(hg_model),sizeof(hg_cfg),offsetof(hg_cfg,heightfield),offsetof(hg_cfg,seed),sizeof(hg_desc));'
                 'printf(" %zu %zu %zu",sizeof(hg_gather_table),offsetof(hg_gather_table,width),'
                 'offsetof(hg_gather_table,dst_dtype));}')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(c), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(N.HgModel), ctypes.sizeof(N.HgCfg), N.HgCfg.heightfield.offset, N.HgCfg.seed.offset,
            ctypes.sizeof(N.HgDesc), ctypes.sizeof(N.GatherTable), N.GatherTable.width.offset,
            N.GatherTable.dst_dtype.offset]
    assert got == want


def test_model_table():
    m, js = N.load_model()
    assert m.num_bodies == 13 and m.num_dof == 12 and m.num_contacts == 24 and m.num_foot_contacts == 8
    assert m.num_leg_contacts == 16 and m.num_capsules == 9 and m.num_pairs == 13
    assert m.num_contacts + m.num_pairs == 37  # > 32: K_step's detection runs its second round
    # ankle pitch / roll joints carry the URDF's 0.1 N m friction; the asset armature is 0
    assert [round(m.joint_friction[b], 6) for b in range(1, 13)] == [0, 0, 0, 0, 0.1, 0.1] * 2
    assert all(m.armature[b] == 0.0 for b in range(13))
    caps = js["capsules"]
    # pairs 0..6: left leg capsule -> right leg capsule, no foot-thigh pair
    for a, b in js["pairs"][:7]:
        assert caps[a]["side"] == "left" and caps[b]["side"] == "right"
        assert {caps[a]["part"], caps[b]["part"]} != {"leg_pitch", "ankle_roll"}
    # then the base-link shapes (body 0) vs the legs: each hand vs its side's thigh and shin, the
    # base-box bottom face (kind 1) vs each thigh; the base shape is always the pair's first
    base_pairs = [(caps[a]["part"], caps[a]["side"], caps[b]["part"], caps[b]["side"]) for a, b in js["pairs"][7:]]
    assert base_pairs == [("hand", "left", "leg_pitch", "left"), ("hand", "left", "knee", "left"),
                          ("hand", "right", "leg_pitch", "right"), ("hand", "right", "knee", "right"),
                          ("box_bottom", "base", "leg_pitch", "left"), ("box_bottom", "base", "leg_pitch", "right")]
    for a, _ in js["pairs"][7:]:
        assert caps[a]["body"] == 0
    assert [m.capsule_kind[k] for k in range(9)] == [0] * 8 + [1]
    # the box face is the base-link box's bottom (XBot-L.urdf:37-42: 0.4 m cube centred 0.1 m up)
    assert caps[8]["p0"] == [-0.2, -0.2, -0.1] and caps[8]["p1"] == [0.2, 0.2, -0.1]
    assert abs(js["total_mass"] - 53.036) < 0.01
    bodies = [b["name"] for b in js["bodies"]]
    assert bodies.index("left_ankle_roll_link") == 6 and bodies.index("right_ankle_roll_link") == 12
    assert bodies.index("left_knee_link") == 4 and bodies.index("right_knee_link") == 10


def test_stacked_image_and_split_gemm_reject_bad_arguments():
    """hg_gemm_x6_image_jobs_pitched and hg_gemm_f32_img_split validate their arguments before any
    device work (CPU: every call here is refused, nothing is launched)."""
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libhgsim.so not built")
    L = N.load_library()
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    fake = vp(0x10000)  # 16-byte aligned, never dereferenced on a refused call
    P, ld, tr = (vp * 1)(fake), (i64 * 1)(705), (ctypes.c_int * 1)(0)
    rows, K, img = (i64 * 1)(128), (i64 * 1)(705), (vp * 1)(fake)
    # pitch rows below the job's rows
    assert L.hg_gemm_x6_image_jobs_pitched(P, ld, tr, rows, K, img, (i64 * 1)(64), 1, None) != 0
    # band chains: a 480 + 32 split would race on rows 480..511 and write past the
    # image; a lone band smaller than its pitch leaves rows nobody writes; a gap between bands
    base = 0x100000

    def bands(rs, addr=None, pitch=None):
        m = len(rs)
        offs = addr or [sum(rs[:i]) for i in range(m)]
        return L.hg_gemm_x6_image_jobs_pitched((vp * m)(*[fake] * m), (i64 * m)(*[705] * m), (ctypes.c_int * m)(*[0] * m),
                                               (i64 * m)(*rs), (i64 * m)(*[705] * m),
                                               (vp * m)(*[vp(base + 32 * o) for o in offs]),
                                               (i64 * m)(*[pitch or sum(rs)] * m), m, None)
    assert bands([480, 32]) != 0
    assert bands([96, 32]) != 0
    assert bands([128], pitch=640) != 0
    assert bands([512, 128], addr=[0, 544]) != 0
    nbytes = L.hg_gemm_x6_image_bytes(640, 705)
    args = dict(A=fake, lda=705, Bimg=fake, bias=fake, bias2=fake, C=fake, ldc=512, C2=fake, ldc2=128, nsplit=512,
                M=24576, N=640, K=705, act=1, tile=25, nbytes=nbytes)

    def call(**kw):
        a = dict(args, **kw)
        return L.hg_gemm_f32_img_split(a["A"], a["lda"], a["Bimg"], a["bias"], a["bias2"], a["C"], a["ldc"], a["C2"],
                                       a["ldc2"], a["nsplit"], a["M"], a["N"], a["K"], a["act"], a["tile"],
                                       a["nbytes"], None)
    assert call(nsplit=500) != 0          # not a multiple of 256
    assert call(nsplit=640) != 0          # no second band
    assert call(bias2=None) != 0          # one bias without the other
    assert call(ldc=256) != 0             # first output narrower than its band
    assert call(nbytes=nbytes - 16) != 0  # image built for another shape
    assert call(tile=5) != 0              # f32 tiles have no image form


def test_splitk_forward_rejects_bad_arguments():
    """hg_gemm_f32_splitk validates its arguments before any device work (CPU: every call here is
    refused, nothing is launched); hg_gemm_splitk_kslice is the slice length it checks against."""
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libhgsim.so not built")
    L = N.load_library()
    assert L.hg_gemm_splitk_kslice(705, 2) == 368
    assert L.hg_gemm_splitk_kslice(705, 4) == 192
    assert L.hg_gemm_splitk_kslice(0, 2) < 0
    fake = ctypes.c_void_p(0x10000)  # 16-byte aligned, never dereferenced on a refused call
    args = dict(A=fake, lda=705, B=fake, ldb=705, bias=fake, C=fake, ldc=512, ws=fake, wsf=2 * 4096 * 512, M=4096,
                N=512, K=705, act=1, tile=21, slices=2)

    def call(**kw):
        a = dict(args, **kw)
        return L.hg_gemm_f32_splitk(a["A"], a["lda"], a["B"], a["ldb"], a["bias"], a["C"], a["ldc"], a["ws"], a["wsf"],
                                    a["M"], a["N"], a["K"], a["act"], a["tile"], a["slices"], None)
    assert call(slices=1) != 0                    # not split
    assert call(slices=17) != 0
    assert call(K=16, lda=16, ldb=16) != 0        # an empty slice (kslice 16: slice 1 starts at K)
    assert call(wsf=2 * 4096 * 512 - 1) != 0      # workspace short of slices x M x N
    assert call(ws=ctypes.c_void_p(0x10004)) != 0  # workspace not 16-byte aligned
    assert call(tile=5) != 0                      # f32 tiles have no split-K form
    assert call(bias=None) != 0
    assert call(ldc=500) != 0
    assert call(act=2) != 0


def test_splitk_img_forward_rejects_bad_arguments():
    """hg_gemm_f32_splitk_img refuses before any device work: an image built for another shape, the
    tiles with two chunks per stage (24, 26, 29), f32 tiles, an empty slice, a short workspace."""
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libhgsim.so not built")
    L = N.load_library()
    fake = ctypes.c_void_p(0x10000)
    nbytes = int(L.hg_gemm_x6_image_bytes(512, 705))
    args = dict(A=fake, lda=705, img=fake, nb=nbytes, bias=fake, C=fake, ldc=512, ws=fake, wsf=4 * 4096 * 512,
                M=4096, N=512, K=705, act=1, tile=25, slices=4)

    def call(**kw):
        a = dict(args, **kw)
        return L.hg_gemm_f32_splitk_img(a["A"], a["lda"], a["img"], a["nb"], a["bias"], a["C"], a["ldc"], a["ws"],
                                        a["wsf"], a["M"], a["N"], a["K"], a["act"], a["tile"], a["slices"], None)
    assert call(nb=nbytes - 16) != 0               # image built for another shape
    for t in (24, 26, 29, 5, 18, 33):
        assert call(tile=t) != 0
    assert call(img=ctypes.c_void_p(0x10004)) != 0  # image not 16-byte aligned
    assert call(K=16, lda=16, nb=int(L.hg_gemm_x6_image_bytes(512, 16))) != 0  # an empty slice
    assert call(wsf=4 * 4096 * 512 - 1) != 0
    assert call(slices=1) != 0
    assert call(bias=None) != 0
    assert call(act=2) != 0
