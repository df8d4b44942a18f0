"""DeepDeform input formats: loaders checked against the reference's example_data files (committed
under tests/golden/deepdeform by make_deepdeform_fixture.py, expected values decoded there with `struct`, the reference's
own method), writer/reader round trips, frame datasets over the DeepDeform layout, and the CPU back-projection oracle
pinned by the reference's float64 loop (image_processing/__init__.py:312-330)."""
import json
import os

import numpy as np
import pytest

from dynamicfuion_python_amd.data import camera as dcam
from dynamicfuion_python_amd.data import frame as dfr
from dynamicfuion_python_amd.data import io as dio

DD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "deepdeform")
SEQ = os.path.join(DD, "test", "seq017")
with open(os.path.join(DD, "expected.json")) as _f:
    EXPECTED = json.load(_f)
GRAPH = EXPECTED["graph"]


def _check_stats(a, exp):
    v = np.asarray(a, np.float64).ravel()
    fin = v[np.isfinite(v)]
    assert v.size == exp["count"] and fin.size == exp["finite"]
    assert fin.sum() == pytest.approx(exp["sum"], rel=1e-9, abs=1e-9)
    assert (fin ** 2).sum() == pytest.approx(exp["sumsq"], rel=1e-9, abs=1e-9)
    k = len(exp["first_row"])
    np.testing.assert_array_equal(v[:k], np.asarray(exp["first_row"], np.float64))
    np.testing.assert_array_equal(v[-k:], np.asarray(exp["last_row"], np.float64))


@pytest.mark.parametrize("kind,loader,shape", [
    ("graph_nodes", dio.load_graph_nodes_or_deformations, lambda h: (h[0], 3)),
    ("graph_edges", dio.load_graph_edges, lambda h: (h[0], h[1])),
    ("graph_edges_weights", dio.load_graph_edges_weights, lambda h: (h[0], h[1])),
    ("graph_clusters", dio.load_graph_clusters, lambda h: (h[0], 1)),
])
def test_graph_files_match_reference_decoding(kind, loader, shape):
    exp = EXPECTED[kind]
    a = loader(os.path.join(SEQ, kind, GRAPH + ".bin"))
    assert a.shape == shape(exp["header"])
    assert a.dtype == (np.float32 if kind in ("graph_nodes", "graph_edges_weights") else np.int32)
    _check_stats(a, exp)


@pytest.mark.parametrize("ext,channels", [("oflow", 2), ("sflow", 3)])
def test_flow_binary_matches_reference_decoding(ext, channels):
    exp = EXPECTED[ext]
    w, h, c = exp["header"]
    flow = dio.load_flow(os.path.join(DD, "flow", f"shirt_000000_000110_rows.{ext}"))
    assert flow.shape == (c, h, w) == (channels, EXPECTED["flow_rows"][1] - EXPECTED["flow_rows"][0], 640)
    v = flow.astype(np.float64).ravel()
    fin = v[np.isfinite(v)]
    assert fin.size == exp["finite"] and fin.sum() == pytest.approx(exp["sum"], rel=1e-9)
    k = len(exp["first_row"])
    np.testing.assert_array_equal(v[:k], np.asarray(exp["first_row"], np.float64))


def test_graph_is_consistent():
    nodes = dio.load_graph_nodes_or_deformations(os.path.join(SEQ, "graph_nodes", GRAPH + ".bin"))
    edges = dio.load_graph_edges(os.path.join(SEQ, "graph_edges", GRAPH + ".bin"))
    weights = dio.load_graph_edges_weights(os.path.join(SEQ, "graph_edges_weights", GRAPH + ".bin"))
    assert edges.shape == weights.shape and edges.shape[0] == nodes.shape[0]
    assert edges.min() >= -1 and edges.max() < nodes.shape[0]
    assert np.all(np.isfinite(nodes)) and np.all(nodes[:, 2] > 0.5)   # metres, in front of the camera
    # weights are zero exactly where there is no edge
    assert np.all((weights == 0) | (edges >= 0))


def test_round_trips(tmp_path):
    rng = np.random.default_rng(3)
    nodes = rng.normal(size=(17, 3)).astype(np.float32)
    edges = rng.integers(-1, 17, size=(17, 8)).astype(np.int32)
    weights = rng.random((17, 8)).astype(np.float32)
    rot = rng.normal(size=(17, 3, 3)).astype(np.float32)
    clusters = rng.integers(0, 4, size=(17, 1)).astype(np.int32)
    cases = [
        (dio.save_graph_nodes, dio.load_graph_nodes_or_deformations, nodes),
        (dio.save_graph_node_deformations, dio.load_graph_nodes_or_deformations, nodes),
        (dio.save_graph_node_translations, dio.load_graph_node_translations, nodes),
        (dio.save_graph_node_rotations, dio.load_graph_node_rotations, rot),
        (dio.save_graph_edges, dio.load_graph_edges, edges),
        (dio.save_graph_edges_weights, dio.load_graph_edges_weights, weights),
        (dio.save_graph_clusters, dio.load_graph_clusters, clusters),
        (dio.save_float_image, dio.load_float_image, rng.random((5, 7, 4)).astype(np.float32)),
        (dio.save_int_image, dio.load_int_image, rng.integers(-1, 99, size=(5, 7, 4)).astype(np.int32)),
        (dio.save_flow, dio.load_flow, rng.normal(size=(2, 6, 9)).astype(np.float32), ".oflow"),
        (dio.save_flow, dio.load_flow, rng.normal(size=(3, 6, 9)).astype(np.float32), ".sflow"),
        (dio.save_flow, dio.load_flow, rng.normal(size=(6, 9, 2)).astype(np.float32), ".flo"),
    ]
    for i, case in enumerate(cases):
        save, load, a = case[:3]
        path = str(tmp_path / f"f{i}{case[3] if len(case) > 3 else '.bin'}")
        save(path, a)
        b = load(path)
        assert b.dtype == a.dtype and b.shape == a.shape, (save.__name__, b.shape)
        np.testing.assert_array_equal(b, a)


@pytest.mark.parametrize("shape", [(6, 9), (6, 9, 3)])
def test_pfm_round_trip(tmp_path, shape):
    a = np.random.default_rng(1).normal(size=shape).astype(np.float32)
    dio.save_PFM(str(tmp_path / "x.pfm"), a)
    b, scale = dio.load_PFM(str(tmp_path / "x.pfm"))
    assert scale == 1.0
    np.testing.assert_array_equal(b, a)
    if len(shape) == 3:
        dio.save_flow(str(tmp_path / "f.pfm"), a)
        np.testing.assert_array_equal(dio.load_flow(str(tmp_path / "f.pfm")), a[:, :, :2])


def test_malformed_files(tmp_path):
    p = tmp_path / "t.bin"
    p.write_bytes(np.asarray([10], "<u4").tobytes() + np.zeros(3 * 9, "<f4").tobytes())   # header says 10 nodes, 9 present
    with pytest.raises(ValueError, match="truncated"):
        dio.load_graph_nodes_or_deformations(str(p))
    p.write_bytes(b"\x01\x00")
    with pytest.raises(ValueError, match="truncated"):
        dio.load_graph_edges(str(p))
    with pytest.raises(FileNotFoundError):
        dio.load_float_image(str(tmp_path / "missing.bin"))
    (tmp_path / "bad.flo").write_bytes(b"XXXX" + bytes(8))
    with pytest.raises(ValueError, match="PIEH"):
        dio.load_flow(str(tmp_path / "bad.flo"))
    with pytest.raises(ValueError, match="extension"):
        dio.load_flow(str(tmp_path / "x.png"))
    (tmp_path / "bad.pfm").write_bytes(b"P6\n")
    with pytest.raises(ValueError, match="PFM"):
        dio.load_PFM(str(tmp_path / "bad.pfm"))
    with pytest.raises(ValueError):
        dio.save_graph_nodes(str(p), np.zeros((4, 2), np.float32))
    with pytest.raises(ValueError):
        dio.save_PFM(str(tmp_path / "y.pfm"), np.zeros((4, 4), np.float64))


def test_empty_graph(tmp_path):
    p = str(tmp_path / "e.bin")
    dio.save_graph_edges(p, np.zeros((0, 8), np.int32))
    assert dio.load_graph_edges(p).shape == (0, 8)
    dio.save_graph_nodes(p, np.zeros((0, 3), np.float32))
    assert dio.load_graph_nodes_or_deformations(p).shape == (0, 3)


def test_images_and_intrinsics(tmp_path):
    depth = dio.load_depth_image(os.path.join(SEQ, "depth", "000300.png"))
    assert depth.dtype == np.uint16 and depth.shape == (480, 640)
    assert 0 < depth.max() < 5000 and (depth > 0).sum() > 100000   # millimetres
    color = dio.load_color_image(os.path.join(SEQ, "color", "000300.jpg"))
    assert color.dtype == np.uint8 and color.shape == (480, 640, 3)
    K = dcam.load_intrinsic_3x3_matrix_from_text_4x4_matrix(os.path.join(SEQ, "intrinsics.txt"))
    assert K.shape == (3, 3) and K[2, 2] == 1.0
    fx, fy, cx, cy = dcam.load_intrinsic_matrix_entries_from_text_4x4_matrix(os.path.join(SEQ, "intrinsics.txt"))
    assert (fx, fy, cx, cy) == (K[0, 0], K[1, 1], K[0, 2], K[1, 2]) == (575.548, 577.46, 323.172, 236.417)
    intr, m4 = dcam.load_open3d_intrinsics_from_text_4x4_matrix_and_image(os.path.join(SEQ, "intrinsics.txt"),
                                                                          os.path.join(SEQ, "depth", "000300.png"))
    assert (intr.width, intr.height) == (640, 480) and m4.shape == (4, 4)
    assert dcam.intrinsic_projection_parameters_as_dict(intr) == {"fx": fx, "fy": fy, "cx": cx, "cy": cy}
    # depth PNG round trip through PIL (uint16 preserved)
    from PIL import Image
    Image.fromarray(depth).save(str(tmp_path / "d.png"))
    np.testing.assert_array_equal(dio.load_depth_image(str(tmp_path / "d.png")), depth)
    dio.save_rgb_image(str(tmp_path / "c.png"), color)
    np.testing.assert_array_equal(dio.load_color_image(str(tmp_path / "c.png")), color)


def test_crop_and_cropped_intrinsics():
    crop = dcam.StaticCenterCrop((480, 640), (448, 640))
    img = np.arange(480 * 640).reshape(480, 640)
    out = crop(img)
    assert out.shape == (448, 640) and out[0, 0] == img[16, 0]
    assert crop(np.zeros((480, 640, 3))).shape == (448, 640, 3)
    # quirk D1: cx gains (w / original_w) / 2 (image_processing/__init__.py:301-309)
    assert dcam.modify_intrinsics_due_to_cropping(500.0, 500.0, 320.0, 240.0, 448, 640) == (500.0, 500.0, 320.5, 224.0)


def test_frame_name_masks():
    assert dfr.make_frame_file_name_mask("frame-000042.color", ".png") == "frame-{:06d}.color.png"
    assert dfr.make_frame_file_name_mask("000300", ".jpg") == "{:06d}.jpg"
    with pytest.raises(ValueError):
        dfr.make_frame_file_name_mask("color", ".png")


def test_frame_pair_and_sequence_over_deepdeform_layout():
    pair = dfr.FramePairDataset(300, 600, 17, dfr.DataSplit.TEST, dfr.DatasetType.LOCAL, base_directory=DD).load()
    assert pair.graph_filename == GRAPH and pair.segment_name == "shirt"
    assert os.path.isfile(pair.get_source_depth_image_path()) and os.path.isfile(pair.get_target_depth_image_path())
    assert os.path.isfile(pair.get_source_color_image_path())
    nodes, edges, weights, deformations, clusters = pair.load_graph_data(GRAPH)
    assert nodes.shape == (109, 3) and edges.shape == (109, 8) and deformations is None and clusters.shape == (109, 1)
    with pytest.raises(ValueError, match="no masks"):
        pair.get_source_mask_image_path()

    seq = dfr.FrameSequenceDataset(17, dfr.DataSplit.TEST, base_dataset_type=dfr.DatasetType.LOCAL, base_directory=DD,
                                   frame_indices=[300, 600]).load()
    assert len(seq) == 2 and seq.resolution == (480, 640)
    assert seq.get_current_graph_name() is None
    f = seq.get_next_frame()
    assert f.frame_index == 300 and seq.get_current_graph_name() == GRAPH
    assert f.load_depth_image_numpy().shape == (480, 640)
    assert f.load_color_image_numpy()[..., ::-1].tolist() == f.load_color_image_rgb().tolist()   # BGR vs RGB
    assert seq.has_more_frames() and seq.get_next_frame().frame_index == 600 and not seq.has_more_frames()
    assert seq.get_current_graph_name() is None and seq.get_next_frame() is None
    seq.rewind()
    assert [fr.frame_index for fr in seq] == [300, 600]
    seq.advance_to_frame(600)
    assert seq.get_next_frame_index() == 600
    with pytest.raises(ValueError):
        seq.advance_to_frame(301)

    unloaded = dfr.FrameSequenceDataset(17, dfr.DataSplit.TEST, base_directory=DD)
    with pytest.raises(ValueError, match="loaded"):
        unloaded.get_next_frame()
    with pytest.raises(ValueError, match="start"):   # consecutive counting from frame 0 finds nothing
        dfr.FrameSequenceDataset(17, dfr.DataSplit.TEST, base_dataset_type=dfr.DatasetType.LOCAL, base_directory=DD).load()
    with pytest.raises(ValueError, match="sequence_id"):
        dfr.FrameSequenceDataset(None, None, base_dataset_type=dfr.DatasetType.LOCAL, base_directory=DD).load()


def test_custom_directory_discovery(tmp_path):
    from PIL import Image
    d = np.zeros((4, 8), np.uint16)
    for i in range(3):
        Image.fromarray(d).save(str(tmp_path / f"depth_{i:04d}.png"))
        Image.fromarray(np.zeros((4, 8, 3), np.uint8)).save(str(tmp_path / f"rgb_{i:04d}.jpg"))
    (tmp_path / "camera_intrinsics.txt").write_text("1 0 2 0\n0 1 2 0\n0 0 1 0\n0 0 0 1\n")
    seq = dfr.FrameSequenceDataset(base_dataset_type=dfr.DatasetType.CUSTOM, custom_frame_directory=str(tmp_path)).load()
    assert len(seq) == 3 and seq.resolution == (4, 8)
    assert seq.get_intrinsics_path().endswith("camera_intrinsics.txt")
    assert seq.get_frame_at(2).get_depth_image_path().endswith("depth_0002.png")
    assert seq.get_current_frame_graph_warp_field() is None
    static = dfr.StaticFrameSequenceDataset(base_dataset_type=dfr.DatasetType.CUSTOM, custom_frame_directory=str(tmp_path),
                                            frame_count=3).load()
    assert static.get_frame_at(2).get_depth_image_path().endswith("depth_0000.png")
    sub = tmp_path / "sub"
    (sub / "depth").mkdir(parents=True)
    (sub / "color").mkdir()
    Image.fromarray(d).save(str(sub / "depth" / "000000.png"))
    Image.fromarray(np.zeros((4, 8, 3), np.uint8)).save(str(sub / "color" / "000000.jpg"))
    s2 = dfr.StandaloneFrameDataset(0, base_dataset_type=dfr.DatasetType.CUSTOM, custom_frame_directory=str(sub)).load()
    assert s2.get_depth_image_path().endswith(os.path.join("depth", "000000.png"))
    with pytest.raises(ValueError, match="custom_frame_directory"):
        dfr.StandaloneFrameDataset(0, base_dataset_type=dfr.DatasetType.CUSTOM).load()


def test_backproject_oracle_against_reference_loop(oracle_mod):
    """oracle.backproject_depth (float32, reference op order) vs the reference's float64 Python loop
    (image_processing/__init__.py:312-330) restated: agreement to float32 rounding."""
    depth = dio.load_depth_image(os.path.join(SEQ, "depth", "000300.png"))[::8, ::8]
    fx, fy, cx, cy = 575.548, 577.46, 323.172 / 8, 236.417 / 8
    got = oracle_mod.backproject_depth(depth, fx, fy, cx, cy, 1000.0)
    H, W = depth.shape
    ref = np.zeros((H, W, 3))
    for y in range(H):
        for x in range(W):
            d = depth[y, x] / 1000.0
            if d > 0:
                ref[y, x] = (d * (x - cx) / fx, d * (y - cy) / fy, d)
    np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-7)
    assert np.all(got[depth == 0] == 0)
    f = oracle_mod.backproject_depth(depth.astype(np.float32) / 1000.0, fx, fy, cx, cy)
    np.testing.assert_allclose(f, ref, rtol=2e-6, atol=1e-7)


def test_fusion_pipeline_switches_fail_loudly():
    """The tracking-method switch (apps/fusion/pipeline.py:356-365): paths this build does not provide raise before any
    GPU work."""
    from dynamicfuion_python_amd import fusion as F
    seq = dfr.FrameSequenceDataset(17, dfr.DataSplit.TEST, base_dataset_type=dfr.DatasetType.LOCAL, base_directory=DD,
                                   frame_indices=[300, 600])
    with pytest.raises(NotImplementedError, match="NEURAL"):
        F.FusionPipeline(seq, F.FusionParameters(tracking_method=F.TrackingMethod.NEURAL))
    with pytest.raises(NotImplementedError, match="FIRST_FRAME_DEPTH_IMAGE"):
        F.FusionPipeline(seq, F.FusionParameters(graph_generation_mode=F.GraphGenerationMode.FIRST_FRAME_DEPTH_IMAGE))
    with pytest.raises(ValueError, match="nodes="):
        F.FusionPipeline(seq, F.FusionParameters(graph_generation_mode=F.GraphGenerationMode.PROVIDED_NODES))
    p = F.FusionParameters()
    assert p.alignment.ndc_convention == 1 and p.alignment.data_term_penalty_function.name == "SQUARE"
