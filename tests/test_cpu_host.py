"""CPU-only checks: the C-ABI library loads and exports every symbol include/ncf_hip.h declares
(no compute calls without a GPU), the ctypes table matches the header, and the host-side mirror of
the reference surface (state_dict keys, constructor, KJT) behaves like the reference."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest
import torch

import _ncf_pkg
from tests.conftest import ROOT, sub

ncf = _ncf_pkg.load()
from ncf_amd import _lib  # noqa: E402

HEADER = os.path.join(ROOT, "include", "ncf_hip.h")


def header_decls():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"^\s*([A-Za-z_][\w\s\*]*?)\b(ncf_\w+)\s*\(([^;]*?)\)\s*;", src, re.M | re.S):
        args = [a.strip() for a in m.group(3).split(",") if a.strip() and a.strip() != "void"]
        decls[m.group(2)] = args
    return decls


def test_header_matches_ctypes_table():
    decls = header_decls()
    assert decls, "no declarations parsed"
    assert set(decls) == set(_lib.SIGNATURES), set(decls) ^ set(_lib.SIGNATURES)
    for name, args in decls.items():
        assert len(args) == len(_lib.SIGNATURES[name][1]), name


def test_library_exports_every_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["bash", os.path.join(ROOT, "build_ext.sh")], check=True)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = set(header_decls()) - syms
    assert not missing, missing
    lib = _lib.load()
    assert lib.ncf_version() == 10000
    assert lib.ncf_last_error() is not None
    # workspace queries are pure host arithmetic
    assert _lib.query("ncf_gemm_splitk_workspace", 256, 64, 4) == 4 * (256 * 64 + 256)
    assert _lib.query("ncf_embedding_bwd_workspace", 20480, 64) > 0


def test_library_build_identity_is_checked(monkeypatch, tmp_path):
    """The library carries the hash of the ctypes table and of the kernel sources it was built
    from (ncf_build_info, _abi.py); _lib.load() refuses a library whose table differs from
    SIGNATURES, or whose sources differ from the ones beside the package (a stale build: the
    r05y fault's first suspect, VERDICT r5 / ADVICE r5)."""
    from ncf_amd import _abi
    lib = _lib.load()
    info = _lib.build_info(lib)
    assert info["abi"] == _abi.abi_hash(_lib.SIGNATURES)
    assert info["src"] == _abi.src_hash()
    _lib.check_build(lib)
    changed = dict(_lib.SIGNATURES)
    changed["ncf_fill_2d"] = (_lib.I32, changed["ncf_fill_2d"][1][:-1])   # one argument fewer
    monkeypatch.setattr(_lib, "SIGNATURES", changed)
    with pytest.raises(_lib.NCFLibraryError, match="C-ABI"):
        _lib.check_build(lib)
    monkeypatch.undo()
    # an edited kernel source without a rebuild
    csrc = tmp_path / "csrc"
    csrc.mkdir()
    for f in _abi.source_files():
        if f.endswith((".hip", ".h")) and os.path.dirname(f) == _abi.CSRC:
            (csrc / os.path.basename(f)).write_bytes(open(f, "rb").read())
    (csrc / "adam.hip").write_bytes((csrc / "adam.hip").read_bytes() + b"\n// edited\n")
    monkeypatch.setattr(_abi, "CSRC", str(csrc))
    monkeypatch.setattr(_abi.src_hash, "__defaults__", (str(csrc),))
    with pytest.raises(_lib.NCFLibraryError, match="stale"):
        _lib.check_build(lib)


def test_code_object_is_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", _lib.LIB_PATH],
                         capture_output=True, text=True)
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob or "gfx950" in out.stdout


def test_launch_tape_records_and_rebases():
    """tapes.py's mechanism on a host-only entry point (ncf_adam_step_scalars writes into a
    host buffer): a recorded call replays with its pointer argument re-based onto another
    buffer (same offset), size queries are not recorded, a call outside the fast path
    invalidates the recording."""
    assert _lib.tapes_available()
    a = np.zeros(32, np.float32)
    b = np.zeros(40, np.float32)
    t = _lib.LaunchTape()
    with t.record((a.ctypes.data, a.nbytes)):
        _lib.call("ncf_adam_step_scalars", 1e-3, 0.9, 0.999, 1e-8, 3, 8, a.ctypes.data)
        _lib.query("ncf_adam_step_scalars", 1e-3, 0.9, 0.999, 1e-8, 3, 8, a.ctypes.data)
    assert t.valid and t.calls == 1 and t.size() == (1, 1, 1)
    t.replay((b.ctypes.data + 32,))
    assert np.array_equal(b[8:], a) and not b[:8].any()
    bad = _lib.LaunchTape()
    with bad.record():
        _lib.call("ncf_adam_step_scalars", 1e-3, 0.9, 0.999, 1e-8, 3, 8,
                  ctypes.c_void_p(a.ctypes.data))        # (a ctypes object: not the fast path)
    assert not bad.valid
    with pytest.raises(RuntimeError):
        bad.replay()


def test_state_dict_keys_and_strict_load(f1):
    m = ncf.AdvancedNCF(8031, 366, 5, 24, 64, 64, 32, [256, 128, 64], 4, 0.2, 4)
    keys = list(m.state_dict().keys())
    gold = list(sub(f1, "sd/").keys())
    assert keys == gold and len(keys) == 62
    sd = {k: torch.from_numpy(v) for k, v in sub(f1, "sd/").items()}
    m2 = ncf.AdvancedNCF(int(f1["cfg"][0]), int(f1["cfg"][1]), 5, 24)
    m2.load_state_dict(sd, strict=True)
    for k, v in m2.state_dict().items():
        assert torch.equal(v, sd[k]), k
    # dense params are views into one flat buffer and survive load_state_dict
    eng = m2.engine
    assert all(eng.is_flat_view(p) for _, p in eng.dense_params())


def test_attribute_surface():
    m = ncf.AdvancedNCF(100, 50, 5, 24)
    # attributes read by trainer.py:567-569, generate_embeddings.py:100-104, app.py:156-184
    for a in ("num_users", "num_products", "mf_embedding_dim", "num_categories",
              "num_departments", "num_heads", "temporal_dim", "negative_samples"):
        assert hasattr(m, a)
    assert m.user_product_attention.scale == pytest.approx(4.0)
    assert tuple(m.final[0].weight.shape) == (1, 2)
    assert hasattr(m.user_product_attention, "q_proj") and hasattr(m.user_product_attention, "k_proj")
    assert tuple(m.temporal_encoding.hour_embed.weight.shape) == (24, 32)
    assert isinstance(m.mlp_norm, torch.nn.LayerNorm)


def test_cpu_forward_fails_loudly():
    m = ncf.AdvancedNCF(10, 10, 5, 24)
    kjt = ncf.KeyedJaggedTensor.from_lengths_sync(
        keys=["user_id", "product_id"], values=torch.tensor([1, 2, 3, 4]),
        lengths=torch.ones(4, dtype=torch.long))
    m.eval()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(kjt)


def test_kjt_surface():
    KJT = ncf.KeyedJaggedTensor
    v = torch.tensor([5, 6, 7, 1, 2, 3])
    k = KJT.from_lengths_sync(keys=["user_id", "product_id"], values=v,
                              lengths=torch.ones(6, dtype=torch.long))
    assert k.keys() == ["user_id", "product_id"]
    d = k.single_id_split()
    assert d["user_id"].tolist() == [5, 6, 7] and d["product_id"].tolist() == [1, 2, 3]
    td = k.to_dict()
    assert td["product_id"].values().tolist() == [1, 2, 3]
    assert k.offsets().tolist() == [0, 1, 2, 3, 4, 5, 6]
    # generate_embeddings.py:107-112 builds it with explicit offsets
    k2 = KJT(keys=["user_id", "product_id"], values=torch.tensor([0, 9]),
             lengths=torch.tensor([1, 1]), offsets=torch.tensor([0, 1, 2]))
    assert k2.single_id_split()["product_id"].tolist() == [9]
    bad = KJT.from_lengths_sync(keys=["user_id", "product_id"], values=torch.tensor([1, 2, 3, 4]),
                                lengths=torch.tensor([2, 0, 1, 1]))
    with pytest.raises(NotImplementedError):
        bad.single_id_split()


def test_to_keeps_flat_layout():
    m = ncf.AdvancedNCF(10, 10, 5, 24)
    w0 = m.mlp[0].weight.detach().clone()
    m = m.double().float()
    assert torch.equal(m.mlp[0].weight.detach(), w0.float())
    assert all(m.engine.is_flat_view(p) for _, p in m.engine.dense_params())


def test_reduce_list_layout_and_scratch_query():
    """ncf_reduce_desc / ncf_reduce_list mirror the header layout; the batch scratch query is
    host arithmetic: one [chunks, L] block per descriptor with P > 256 partials (64 per chunk;
    up to 256 reduce in one stage)."""
    import ctypes
    assert ctypes.sizeof(_lib.ReduceDesc) == 56
    assert ctypes.sizeof(_lib.ReduceList) == 8 + 56 * _lib.REDUCE_LIST_MAX
    src = open(HEADER).read()
    assert f"#define NCF_REDUCE_LIST_MAX {_lib.REDUCE_LIST_MAX}" in src
    lst = _lib.ReduceList()
    for P, L in ((100, 33), (256, 4096), (260, 512), (1024, 768)):
        d = lst.d[lst.count]
        d.part, d.out, d.stride, d.ldo, d.L, d.cols, d.P, d.scale = 8, 8, L, L, L, L, P, 1.0
        lst.count += 1
    assert _lib.query("ncf_reduce_batch_scratch", lst.address) == 5 * 512 + 16 * 768
    empty = _lib.ReduceList()
    assert _lib.load().ncf_reduce_batch(empty.address, None, 0, None) == 0  # nothing to launch


# ----------------------------------------------------------------------------- 8f: negatives
def test_inverse_popularity_weights_vs_oracle():
    from oracle import ncf_oracle as O
    from ncf_amd.data import inverse_popularity_weights
    g = torch.Generator().manual_seed(3)
    prods = torch.randint(0, 37, (500,), generator=g)
    prods[prods == 5] = 6                      # product 5 never seen: count clamps to 1
    np.testing.assert_allclose(inverse_popularity_weights(prods, 40),
                               O.inverse_popularity_weights(prods.tolist(), 40), rtol=1e-12)


@pytest.mark.parametrize("n", [1, 2, 7, 1000])
def test_alias_table_reconstructs_weights(n):
    """ncf_alias_build (host code in libncf_hip.so): each item's total mass over the table,
    (prob[i] + sum_{alias[j] = i} (1 - prob[j])) / n, equals its normalised weight."""
    from ncf_amd.data import alias_table
    rng = np.random.default_rng(n)
    w = rng.random(n) ** 3
    w[rng.random(n) < 0.1] = 0.0
    if w.sum() == 0:
        w[0] = 1.0
    prob, alias = alias_table(w)
    assert prob.min() >= 0 and prob.max() <= 1 and alias.min() >= 0 and alias.max() < n
    mass = prob.astype(np.float64).copy()
    np.add.at(mass, alias, 1.0 - prob.astype(np.float64))
    np.testing.assert_allclose(mass / n, w / w.sum(), atol=1e-6)


def test_negative_distribution_oracle_cases():
    from oracle import ncf_oracle as O
    w = np.array([0.1, 0.2, 0.3, 0.4])
    d = O.negative_distribution(w, [], 0)           # only the positive is rejected
    assert d[0] == 0 and abs(d.sum() - 1) < 1e-12
    d = O.negative_distribution(w, [0, 1, 2, 3], 2)  # bought everything: any but the positive
    np.testing.assert_allclose(d, [1 / 3, 1 / 3, 0, 1 / 3])


# ----------------------------------------------------------------------------- 8f: ANN export
def test_product_index_and_distinct_rows():
    from ncf_amd.export import distinct_products, product_index
    assert product_index("P1A", 366) == 26 and product_index("ff", 100) == 55
    assert product_index("P0", 7) == 0
    rows = [{"product_id": "P10"}, {"product_id": None}, {"category_id": "x"},
            {"product_id": "P10"}, {"product_id": "P2F"}]
    assert distinct_products(rows, 366) == (["P10", "P2F"], [16, 47])


def test_embeddings_jsonl_format():
    import io
    import json
    from ncf_amd.export import write_embeddings_jsonl
    e = torch.tensor([[0.6, 0.8], [1.0, 0.0]])
    buf = io.StringIO()
    assert write_embeddings_jsonl(buf, ["P1", "P2"], e) == 2
    lines = buf.getvalue().splitlines()
    assert lines[0].startswith('{"id": "P1", "embedding": [')
    rec = [json.loads(x) for x in lines]
    assert rec[1] == {"id": "P2", "embedding": [1.0, 0.0]}
    assert rec[0]["embedding"] == [float(np.float32(0.6)), float(np.float32(0.8))]


# ----------------------------------------------------------------------------- 8f: checkpoints
def test_load_unzipped_archive_roundtrip(tmp_path):
    """An extracted torch.save archive (the layout of the reference's demo model directory) is
    read back through weights_only loading with its own keys, shapes and strides."""
    import zipfile
    from collections import OrderedDict
    from ncf_amd.checkpoint import load_unzipped_archive
    g = torch.Generator().manual_seed(0)
    base = torch.randn(6, 4, generator=g)
    sd = OrderedDict([("a.weight", torch.randn(3, 5, generator=g)), ("b", base),
                      ("c.t", base.t()), ("d", torch.arange(7))])
    f = tmp_path / "m.pt"
    torch.save(sd, f)
    out = tmp_path / "unzipped"
    with zipfile.ZipFile(f) as z:
        root = z.namelist()[0].split("/")[0]
        z.extractall(tmp_path / "x")
    os.rename(tmp_path / "x" / root, out)
    got = load_unzipped_archive(str(out))
    assert list(got) == list(sd)
    for k in sd:
        assert torch.equal(got[k], sd[k]) and got[k].stride() == sd[k].stride()


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/inference/demo/train_20241225_002713_model"),
                    reason="reference checkout not present")
def test_load_reference_demo_directory():
    """The reference's own unzipped demo checkpoint (consolidate_shards.py's input) loads with
    all 62 keys in order and the AdvancedNCF shapes (safe loader; container-only check)."""
    from ncf_amd.checkpoint import load_unzipped_archive
    sd = load_unzipped_archive("/root/reference/src/inference/demo/train_20241225_002713_model")
    assert len(sd) == 62 and list(sd)[0] == "mf_norm.weight"
    assert sd["mf_embedding_collection.embedding_bags.user_id.weight"].shape == (8031, 64)
    assert sd["mlp.0.weight"].shape == (256, 96)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_row_shards_roundtrip(world):
    from collections import OrderedDict
    from ncf_amd.checkpoint import TABLE_KEYS, consolidate_row_shards, shard_state_dict
    g = torch.Generator().manual_seed(world)
    U, I, D = 11, 7, 4
    full = OrderedDict()
    for k in TABLE_KEYS:
        full[k] = torch.randn(U if ".user_id." in k else I, D, generator=g)
    full["mlp.0.weight"] = torch.randn(5, 3, generator=g)
    shards = [shard_state_dict(full, world, r) for r in range(world)]
    assert shards[0][TABLE_KEYS[0]].shape == (-(-U // world), D)
    back = consolidate_row_shards(shards, world, U, I)
    assert list(back) == list(full)
    for k in full:
        assert torch.equal(back[k], full[k])


def test_consistent_batch_sampler_vs_reference():
    """ncf_amd.data.ConsistentBatchSampler against the reference's own batches (F9,
    src/model/data_prep.py:397-443): sizes, last-batch padding with repeats of that batch (still
    short when it holds under half a batch), np.random.shuffle order under the same seed."""
    from ncf_amd.data import ConsistentBatchSampler
    d = np.load(os.path.join(ROOT, "tests", "golden", "f9_batches.npz"))
    idx, bounds = d["indices"], d["bounds"]
    b = 0
    for size, bs, shuffle, nb in d["cases"].tolist():
        if shuffle:
            np.random.seed(size * 100 + bs)
        sm = ConsistentBatchSampler(size, bs, shuffle=bool(shuffle))
        got = list(iter(sm))
        assert len(sm) == nb == len(got)
        for g in got:
            assert g == idx[bounds[b]:bounds[b + 1]].tolist(), (size, bs, shuffle)
            b += 1
    assert b == len(bounds) - 1


def test_struct_mirrors_match_header_layouts():
    """ctypes mirrors of ncf_mlp_layer / ncf_table_pair: every field 8 bytes, header order."""
    import ctypes
    assert ctypes.sizeof(_lib.MlpLayer) == 14 * 8
    assert [f[0] for f in _lib.MlpLayer._fields_] == ["w", "ldw", "b", "gamma", "beta", "r", "a",
                                                       "mean", "rstd", "dlin", "dbias", "dgamma",
                                                       "dbeta", "dw"]
    assert ctypes.sizeof(_lib.TablePair) == 12 * 8
    body = hdr_pair = open(os.path.join(ROOT, "include", "ncf_hip.h")).read()
    body = hdr_pair[hdr_pair.index("typedef struct ncf_table_pair"):hdr_pair.index("} ncf_table_pair;")]
    assert re.findall(r"(\w+)[,;]", body) == [f[0] for f in _lib.TablePair._fields_]
    hdr = open(os.path.join(ROOT, "include", "ncf_hip.h")).read()
    body = hdr[hdr.index("typedef struct ncf_mlp_layer"):hdr.index("} ncf_mlp_layer;")]
    names = re.findall(r"\*?\s*(\w+);", body)
    assert names == [f[0] for f in _lib.MlpLayer._fields_]


def test_shard_struct_mirrors_match_header():
    """ctypes mirrors of ncf_shard_plan_out (12 pointers, header order) and ncf_shard_recv
    (world, start[W_MAX + 1], n0[W_MAX] int32) as include/ncf_hip.h declares them."""
    import ctypes
    hdr = open(os.path.join(ROOT, "include", "ncf_hip.h")).read()
    body = hdr[hdr.index("typedef struct ncf_shard_plan_out"):hdr.index("} ncf_shard_plan_out;")]
    names = re.findall(r"\*\s*(\w+);", body)
    assert names == [f[0] for f in _lib.ShardPlanOut._fields_]
    assert ctypes.sizeof(_lib.ShardPlanOut) == 16 * 8
    wmax = int(re.search(r"#define NCF_SHARD_MAX_WORLD (\d+)", hdr).group(1))
    assert wmax == _lib.SHARD_MAX_WORLD
    assert ctypes.sizeof(_lib.ShardRecv) == 4 * (1 + (wmax + 1) + wmax)
    assert [f[0] for f in _lib.ShardRecv._fields_] == ["world", "start", "n0"]


def test_optimizer_hide_and_restore_param_groups():
    """optim._hide takes the fused step's parameters out of torch's param groups for the
    duration of its own step and the post hook restores them (host logic, no GPU)."""
    from ncf_amd import optim as O
    ps = [torch.nn.Parameter(torch.zeros(3)) for _ in range(5)]
    opt = torch.optim.Adam([{"params": ps[:3]}, {"params": ps[3:]}], lr=1e-3)
    before = [list(g["params"]) for g in opt.param_groups]
    hk = frozenset(id(p) for p in ps[:4])
    for _ in range(2):          # (the second call takes the cached lists)
        O._hide(opt, hk)
        assert [len(g["params"]) for g in opt.param_groups] == [0, 1]
        assert opt.param_groups[1]["params"][0] is ps[4]
        O._restore_groups(opt)
        assert [list(g["params"]) for g in opt.param_groups] == before
