"""Known-answer vectors transcribed from the reference's C++ tests (inputs and expected outputs only)."""
import numpy as np

# cpp/tests/test_rodrigues.cpp:31-53 (AllClose rtol 1e-3, atol 1e-7)
RODRIGUES_AXIS_ANGLE = np.array([[0.16959796, 0.84415948, 0.63673575],
                                 [-0.41038024, -0.41038024, 1.53155991],
                                 [-0.35169471, -1.30855167, 1.67691329]], np.float32)
RODRIGUES_EXPECTED = np.array([[[0.49240388, -0.45682599, 0.74084306], [0.58682409, 0.80287234, 0.10504046], [-0.64278761, 0.38302222, 0.66341395]],
                               [[0., -0.8660254, -0.5], [1., 0., 0.], [0., -0.5, 0.8660254]],
                               [[-0.51100229, -0.49471846, -0.70294402], [0.80211293, 0.01955087, -0.59685225],
                                [0.30901699, -0.86883336, 0.38682953]]], np.float32)

# cpp/tests/test_mesh_warping.cpp:68-87 (warped vertex positions after a -90 deg rotation about Y, AllClose 1e-5)
WARP_EXPECTED_POSITIONS = np.array([[-0., -0.5, -0.5], [-0., 0.5, -0.5], [0., -0.5, 0.5], [0., 0.5, 0.5], [-0., 0., -0.5],
                                    [0., 0., 0.], [0., -0.5, 0.], [0., 0.5, 0.], [0., 0., 0.5]], np.float32)
WARP_EXPECTED_NORMALS = np.tile(np.array([[-1., 0., 0.]], np.float32), (9, 1))

# cpp/tests/test_graph_warp_field.cpp:36-82 (33 nodes, coverage 0.25, 3 layers, radii 2^i * coverage)
HIERARCHY_NODES = np.array([
    [2.11, 3.2, 1], [2.32, 3.7, 1], [2.66, 3.35, 1], [3.36, 3.7, 1], [2.31, 2.75, 1], [2.41, 2.2, 1], [2.71, 2.7, 1], [3.31, 2.8, 1],
    [3.71, 2.8, 1], [3.16, 2.3, 1], [3.56, 2.3, 1], [4.21, 3.7, 1], [4.26, 1.65, 1], [4.61, 1.3, 1], [4.00, 1.0, 1], [3.21, 1.25, 1],
    [2.21, 1.65, 1], [2.36, 1.15, 1], [2.76, 1.75, 1], [2.30, 0.35, 1], [5.71, 0.8, 1], [5.11, 0.65, 1], [5.11, 0.4, 1], [5.51, 0.4, 1],
    [5.91, 0.25, 1], [5.16, 3.25, 1], [5.46, 3.65, 1], [5.71, 3.3, 1], [5.46, 2.75, 1], [5.31, 2.45, 1], [5.51, 2.2, 1], [4.41, 2.65, 1],
    [4.62, 0.3, 1]], np.float32)
HIERARCHY_LAYER0 = sorted([0, 2, 5, 6, 7, 8, 9, 12, 14, 17, 18, 20, 21, 22, 24, 25, 27, 28, 30])          # :84-141
HIERARCHY_LAYER1 = sorted([16, 19, 1, 3, 10, 11, 29, 26, 13, 23])                                     # :145-166
HIERARCHY_LAYER2 = sorted([4, 15, 31, 32])                                                            # :170-176
HIERARCHY_EDGE_SOURCES = [v for v in range(28, -1, -1) for _ in range(4)]                             # :187-192
HIERARCHY_EDGES_ORIGINAL = [                                                                          # :204-321
    (0, 1), (0, 3), (0, 10), (0, 16), (1, 4), (1, 15), (1, 31), (1, 32), (2, 1), (2, 3), (2, 10), (2, 11), (3, 4), (3, 15), (3, 31),
    (3, 32), (5, 1), (5, 3), (5, 10), (5, 16), (6, 1), (6, 3), (6, 10), (6, 16), (7, 1), (7, 3), (7, 10), (7, 11), (8, 3), (8, 10),
    (8, 11), (8, 29), (9, 1), (9, 3), (9, 10), (9, 16), (10, 4), (10, 15), (10, 31), (10, 32), (11, 4), (11, 15), (11, 31), (11, 32),
    (12, 10), (12, 13), (12, 23), (12, 29), (13, 4), (13, 15), (13, 31), (13, 32), (14, 10), (14, 13), (14, 19), (14, 23), (16, 4),
    (16, 15), (16, 31), (16, 32), (17, 10), (17, 13), (17, 16), (17, 19), (18, 10), (18, 13), (18, 16), (18, 19), (19, 4), (19, 15),
    (19, 31), (19, 32), (20, 10), (20, 13), (20, 23), (20, 29), (21, 10), (21, 13), (21, 23), (21, 29), (22, 10), (22, 13), (22, 23),
    (22, 29), (23, 4), (23, 15), (23, 31), (23, 32), (24, 10), (24, 13), (24, 23), (24, 29), (25, 3), (25, 11), (25, 26), (25, 29),
    (26, 4), (26, 15), (26, 31), (26, 32), (27, 11), (27, 13), (27, 26), (27, 29), (28, 11), (28, 13), (28, 26), (28, 29), (29, 4),
    (29, 15), (29, 31), (29, 32), (30, 13), (30, 23), (30, 26), (30, 29)]

# cpp/tests/test_linalg_cholesky.cpp:38-102 (SolveBlockDiagonalCholesky, 3 blocks of 6x6, 2 right-hand sides; AllClose defaults)
CHOLESKY_A = np.array([
    [7.66466999, 7.42160096, 7.96971846, 5.41618416, 5.48901906, 6.29302529], [7.42160096, 11.28136639, 10.02191478, 7.6142696, 6.11965727, 8.29031205],
    [7.96971846, 10.02191478, 12.84076044, 7.99068493, 7.71414652, 8.53580411], [5.41618416, 7.6142696, 7.99068493, 8.59449478, 5.25876695, 6.28306648],
    [5.48901906, 6.11965727, 7.71414652, 5.25876695, 6.5656741, 5.7888223], [6.29302529, 8.29031205, 8.53580411, 6.28306648, 5.7888223, 8.58118284],
    [11.02955047, 7.99694855, 8.60120371, 7.94013951, 8.92082018, 6.28801604], [7.99694855, 9.59915016, 8.38727439, 7.69725731, 8.57161899, 6.67614202],
    [8.60120371, 8.38727439, 10.27710871, 7.29562432, 9.01899879, 6.63105238], [7.94013951, 7.69725731, 7.29562432, 9.06157844, 8.29751497, 5.44649512],
    [8.92082018, 8.57161899, 9.01899879, 8.29751497, 11.55352825, 6.84668649], [6.28801604, 6.67614202, 6.63105238, 5.44649512, 6.84668649, 6.56172847],
    [9.76694034, 7.01864966, 6.48232141, 7.00072462, 7.35419513, 5.94435122], [7.01864966, 9.59364701, 6.5592933, 7.44435127, 7.66117909, 6.28624863],
    [6.48232141, 6.5592933, 10.01902388, 6.28058687, 7.16248224, 6.99130877], [7.00072462, 7.44435127, 6.28058687, 8.7593816, 8.17335754, 6.52806757],
    [7.35419513, 7.66117909, 7.16248224, 8.17335754, 11.15212005, 6.81745422], [5.94435122, 6.28624863, 6.99130877, 6.52806757, 6.81745422, 9.11671782],
], np.float32).reshape(3, 6, 6)
CHOLESKY_B = np.array([[0.45293155, 0.52475495], [0.21761689, 0.54381511], [0.17009712, 0.00117492], [0.72334337, 0.83178217],
                       [0.82902052, 0.62671342], [0.59249606, 0.7532337], [0.41178043, 0.74776442], [0.32215233, 0.54746278],
                       [0.37314376, 0.05380477], [0.06205624, 0.37561555], [0.77131601, 0.40215776], [0.02648144, 0.15254462],
                       [0.80500491, 0.25057921], [0.21371886, 0.43475709], [0.39716974, 0.15878393], [0.1928535, 0.65798109],
                       [0.46133341, 0.05955819], [0.95671584, 0.59674103]], np.float32)
CHOLESKY_X = np.array([[0.03432138, 0.05864467], [-0.09385886, 0.00502414], [-0.26434026, -0.35847137], [0.13916333, 0.15648315],
                       [0.30488228, 0.21968781], [0.0899299, 0.13371622], [0.05101893, 0.18088418], [0.10856187, 0.21007842],
                       [-0.02048628, -0.2150583], [-0.19654963, -0.09012525], [0.22811848, 0.03767047], [-0.20948814, -0.1110012],
                       [0.15458118, -0.03555937], [-0.06289044, 0.00555059], [-0.078527, -0.04738612], [-0.18840044, 0.211494],
                       [0.04203119, -0.14935129], [0.21120842, 0.08139612]], np.float32)

# ---- cpp/tests/test_non_rigid_surface_voxel_block_grid.cpp (TSDF voxel block grid) ----
# :60-111 GetBoundingBoxesOfWarpedBlocks: keys, voxel 0.1, resolution 10, 4 nodes (coverage 1.0, 4 anchors, 0 minimum,
# fixed coverage), every node translated by +1 x; expected boxes (AllClose defaults)
VBG_BOX_KEYS = np.array([[0, 0, 0], [0, 1, 0], [0, 0, 1], [0, 1, 1]], np.int32)
VBG_BOX_NODES = np.array([[0.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0], [0.0, 1.0, 1.0]], np.float32)
VBG_BOX_VOXEL_SIZE, VBG_BOX_RESOLUTION, VBG_BOX_COVERAGE = 0.1, 10, 1.0
VBG_BOX_TRANSLATION = np.array([1.0, 0.0, 0.0], np.float32)
VBG_BOX_EXPECTED = np.array([[1, 0, 0, 2, 1, 1], [1, 1, 0, 2, 2, 1], [1, 0, 1, 2, 1, 2], [1, 1, 1, 2, 2, 2]], np.float32)
# :125-159 GetAxisAlignedBoxesInterceptingSurfaceMask: boxes, 4x4 float depth, K (1, 1, 2, 2), scale 1, max 100,
# stride 1, truncation 0.5
VBG_MASK_BOXES = np.array([[3, 0, 0, 4, 1, 1], [3, 1, 0, 4, 2, 1], [1, 0, 1, 2, 1, 2], [1, 1, 1, 2, 2, 2]], np.float32)
VBG_MASK_DEPTH = np.array([[1.0, 1.0, 0.0, 0.0], [1.0, 1.0, 0.0, 0.0], [0.0, 0.0, 1.2, 1.2], [0.0, 0.0, 1.2, 1.2]], np.float32)
VBG_MASK_K = np.array([[1.0, 0.0, 2.0], [0.0, 1.0, 2.0], [0.0, 0.0, 1.0]])
VBG_MASK_EXPECTED = np.array([False, False, True, True])
# :229-341 IntegrateNonRigid: voxel 0.01, resolution 8, 128 blocks, tsdf f32 / weight u16 / color u16 [3]; 100x100 plane
# at 50 mm (uint16), color 100; K (100, 100, 50, 50); trunc multiplier 2, scale 1000, max 3.0; 5 nodes, node 0 moved
# -1 cm in z, coverage 0.005, threshold on, 4 anchors, minimum 1; hemisphere pinch radius 20 px, +10 mm at the centre;
# block (0, 0, 1) activated; expected ExtractVoxelValuesAt rows (AllClose rtol 1e-5, atol 5e-6)
VBG_NR_NODES = np.array([[0.0, 0.0, 0.05], [0.02, 0.0, 0.05], [-0.02, 0.0, 0.05], [0.0, 0.02, 0.05], [0.0, -0.02, 0.05]], np.float32)
VBG_NR_NODE0_TRANSLATION = np.array([0.0, 0.0, -0.01], np.float32)
VBG_NR_QUERIES = np.array([[0, 0, 5], [1, 0, 5], [0, 1, 5], [2, 0, 5], [0, 2, 5], [0, 1, 6], [0, 0, 6], [0, 0, 4]], np.int32)
VBG_NR_EXPECTED = np.array([
    [0.0, 0.0, 0.05, 0.5, 1.0, 100.0, 100.0, 100.0],
    [0.01, 0.0, 0.05, 0.125, 1.0, 100.0, 100.0, 100.0],
    [0.0, 0.01, 0.05, 0.125, 1.0, 100.0, 100.0, 100.0],
    [0.02, 0.0, 0.05, 0.0, 1.0, 100.0, 100.0, 100.0],
    [0.0, 0.02, 0.05, 0.0, 1.0, 100.0, 100.0, 100.0],
    [0.0, 0.01, 0.06, -0.5, 1.0, 100.0, 100.0, 100.0],
    [0.0, 0.0, 0.06, 0.0, 1.0, 100.0, 100.0, 100.0],
    [0.0, 0.0, 0.04, 0.5, 1.0, 100.0, 100.0, 100.0]], np.float32)

# ---- cpp/tests/test_anchor_computation.cpp:30-83 (Euclidean, variable node weight; 2 nodes for 4 anchors: two slots stay
# empty). Weights and anchors each sorted descending before comparison (AllClose rtol 1e-3, atol 1e-6) ----
ANCHOR_VAR_VERTICES = np.array([[-0.0625, 0.3625, 0.], [-0.0625, 0.2375, 0.], [0.0625, 0.3625, 0.], [0.0625, 0.2375, 0.],
                                [-0.0625, -0.2375, 0.], [-0.0625, -0.3625, 0.], [0.0625, -0.2375, 0.], [0.0625, -0.3625, 0.]], np.float32)
ANCHOR_VAR_NODES = np.array([[0.0, 0.3, 0.0], [0.0, -0.3, 0.0]], np.float32)
ANCHOR_VAR_NODE_WEIGHTS = np.array([0.36, 0.36], np.float32)
ANCHOR_VAR_ANCHORS_SORTED = np.tile(np.array([[1, 0, -1, -1]], np.int32), (8, 1))
_w_near, _w_far = [0.64660899, 0.35339101, 0., 0.], [0.59768616, 0.40231384, 0., 0.]
ANCHOR_VAR_WEIGHTS_SORTED = np.array([_w_near, _w_far, _w_near, _w_far, _w_far, _w_near, _w_far, _w_near], np.float32)

# ---- cpp/tests/test_unproject_3d_points.cpp:30-78: uint16 4x4 depth, K (100, 100, 2, 2), identity extrinsics, scale 1000,
# max 3 (AllClose defaults: rtol 1e-5, atol 1e-8), both layouts ----
UNPROJECT_K = np.array([[100., 0., 2.], [0., 100., 2.], [0., 0., 1.]])
UNPROJECT_DEPTH = np.array([[0, 1000, 2000, 0], [0, 500, 1500, 0], [500, 550, 600, 650], [0, 20, 4000, 0]], np.uint16)
UNPROJECT_POINTS = np.array([
    [0., 0., 0.], [-0.01, -0.02, 1.], [0., -0.04, 2.], [0., 0., 0.],
    [0., 0., 0.], [-0.005, -0.005, 0.5], [0., -0.015, 1.5], [0., 0., 0.],
    [-0.01, 0., 0.5], [-0.0055, 0., 0.55], [0., 0., 0.6], [0.0065, 0., 0.65],
    [0., 0., 0.], [-0.0002, 0.0002, 0.02], [0., 0., 0.], [0., 0., 0.]], np.float32)
UNPROJECT_MASK = np.array([False, True, True, False, False, True, True, False, True, True, True, True, False, True, False, False])

# ---- cpp/tests/test_matmul3d.cpp:29-68: batch of three 2x3 @ 3x2 (margin 1e-6) ----
MATMUL3D_A = np.array([7., 2., 1., 5., 4., 4., 2., 9., 7., 2., 8., 7., 1., 1., 2., 9., 6., 0.], np.float32).reshape(3, 2, 3)
MATMUL3D_B = np.array([9., 4., 6., 9., 5., 10., 2., 6., 3., 6., 5., 1., 6., 4., 7., 4., 2., 5.], np.float32).reshape(3, 3, 2)
MATMUL3D_C = np.array([80., 56., 89., 96., 66., 73., 63., 67., 17., 18., 96., 60.], np.float32).reshape(3, 2, 2)

# ---- cpp/tests/test_extract_face_vertices.cpp:72-100: [XY plane (1.2615, (0,0,1), 4 subdivisions), sphere (0.4, (0,0,0.5), 32)]
# at 640x480, fx = fy = 580, near 0, far 2; 1994 faces kept; the reference compares the mask and the first 334 faces
# (AllClose defaults). Fixture arrays: reference_fixtures/extracted_face_{vertices,mask}_multiple_meshes.npy ----
MULTI_MESH_KEPT = 1994
MULTI_MESH_COMPARED_FACES = 334

# ---- cpp/tests/test_normals_operations.cpp:113-136: red_shorts_200_depth.png (uint16 mm) with red_shorts_intrinsics.txt ->
# ordered point-cloud normals; fixture reference_fixtures/red_shorts_200_normals.npy [480,640,3] ----
RED_SHORTS_K = np.array([[575.548, 0., 323.172], [0., 577.46, 236.417], [0., 0., 1.]])

# ---- cpp/tests/test_linalg_block_routines.cpp:158-190: InvertPositiveSemidefiniteBlocks on three 3x3 SPD blocks
# (AllClose(gt, 1e-4): rtol 1e-4) ----
INVERT_PSD_BLOCKS = np.array([16, 20, 24, 20, 29, 36, 24, 36, 46,
                              100, 110, 120, 110, 185, 204, 120, 204, 274,
                              256, 272, 288, 272, 485, 516, 288, 516, 718], np.float32).reshape(3, 3, 3)
INVERT_PSD_BLOCKS_GT = np.array([0.59375, -0.875, 0.375, -0.875, 2.5, -1.5, 0.375, -1.5, 1.,
                                 0.02893495, -0.01804847, 0.00076531, -0.01804847, 0.04145408, -0.02295918, 0.00076531, -0.02295918,
                                 0.02040816,
                                 0.00966704, -0.00550583, 0.00007925, -0.00550583, 0.0118947, -0.00633981, 0.00007925, -0.00633981,
                                 0.00591716], np.float32).reshape(3, 3, 3)

# ---- cpp/tests/test_linalg_matmul_block_sparse.cpp:30-220: MatmulBlockSparseRowWise / RowWisePadded (AllClose defaults) ----
ROWWISE_A = np.arange(27, 0, -1, dtype=np.float32).reshape(3, 3, 3)
ROWWISE_B = np.concatenate([np.arange(0, 18), np.arange(27, 108)]).astype(np.float32).reshape(11, 3, 3)
ROWWISE_B_COORDS = np.array([[0, 0], [1, 0], [3, 0], [0, 1], [1, 1], [2, 1], [3, 1], [0, 2], [1, 2], [2, 2], [3, 2]], np.int32)
ROWWISE_C = np.array([228, 306, 384, 201, 270, 339, 174, 234, 294,
                      606, 657, 708, 498, 540, 582, 390, 423, 456,
                      3036, 3114, 3192, 2685, 2754, 2823, 2334, 2394, 2454,
                      2442, 2493, 2544, 2010, 2052, 2094, 1578, 1611, 1644,
                      1362, 1386, 1410, 849, 864, 879, 336, 342, 348,
                      5844, 5922, 6000, 5169, 5238, 5307, 4494, 4554, 4614,
                      4278, 4329, 4380, 3522, 3564, 3606, 2766, 2799, 2832,
                      2226, 2250, 2274, 1389, 1404, 1419, 552, 558, 564], np.float32).reshape(8, 3, 3)
ROWWISE_C_COORDS = np.array([[0, 0], [1, 0], [0, 1], [1, 1], [2, 1], [0, 2], [1, 2], [2, 2]], np.int32)
ROWWISE_PADDED_ZERO_BLOCKS = (2, 6, 10)   # the padded result is ROWWISE_C with zero blocks inserted at these indices

# ---- test_linalg_matmul_block_sparse.cpp:233-386: MatmulBlockSparse with int16 breadboards (-1 = empty) ----
MBS_A = np.array([3, 4, 5, 6, 1, 2, 3, 4, 5, 6, 7, 8], np.float32).reshape(3, 2, 2)
MBS_A_BOARD = np.array([[0, 1, -1], [-1, -1, 2]], np.int16)
MBS_B = np.array([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 0], np.float32).reshape(3, 2, 2)
MBS_B_BOARD = np.array([[0, -1], [-1, 1], [2, -1]], np.int16)
# (lhs, transpose lhs, rhs, transpose rhs) -> (blocks, coordinates)
MBS_CASES = {
    "AB": (("A", 0, "B", 0), np.array([15, 22, 23, 34, 19, 22, 43, 50, 111, 50, 151, 70], np.float32).reshape(3, 2, 2),
           np.array([[0, 0], [0, 1], [1, 0]], np.int32)),
    "BtAt": (("B", 1, "A", 1), np.array([15, 23, 22, 34, 111, 151, 50, 70, 19, 43, 22, 50], np.float32).reshape(3, 2, 2),
             np.array([[0, 0], [0, 1], [1, 0]], np.int32)),
    "BtB": (("B", 1, "B", 0), np.array([212, 104, 104, 120, 74, 86, 86, 100], np.float32).reshape(2, 2, 2),
            np.array([[0, 0], [1, 1]], np.int32)),
    "AAt": (("A", 0, "A", 1), np.array([30, 50, 50, 86, 61, 83, 83, 113], np.float32).reshape(2, 2, 2),
            np.array([[0, 0], [1, 1]], np.int32)),
}

# ---- test_linalg_matmul_block_sparse.cpp:398-486: BlockSparseAndVectorProduct (m = 4), NONE with A, TRANSPOSE with B ----
BSV_A_COORDS = np.array([[0, 0], [0, 1], [1, 2]], np.int32)
BSV_B_COORDS = np.array([[0, 0], [1, 1], [2, 0]], np.int32)
BSV_V = np.array([-2, -1, 0, 1, 2, 3], np.float32)
BSV_C = np.array([-8, -12, 28, 38], np.float32)
BSV_D = np.array([46, 12, 7, 8], np.float32)

# ---- test_linalg_matmul_block_sparse.cpp:499-531: DiagonalBlockSparseAndVectorProduct ----
DBSV_D = np.array([2, -3, 2, 2, 1, 1, 4, 2, 4, 3, 6, 3], np.float32).reshape(3, 2, 2)
DBSV_C = np.array([-1, -6, 1, 2, 17, 21], np.float32)

# ---- cpp/tests/test_linalg_block_routines.cpp:32-154: InvertTriangularBlocks (AllClose rtol 1e-4), TransposeBlocksInPlace ----
TRI_LOWER = np.array([1, 0, 0, 2, 3, 0, 4, 5, 6, 7, 0, 0, 8, 9, 0, 10, 11, 12, 13, 0, 0, 14, 15, 0, 16, 17, 18], np.float32).reshape(3, 3, 3)
TRI_LOWER_INV = np.array([1., -0., 0., -0.6666667, 0.33333334, -0., -0.11111111, -0.2777778, 0.16666667,
                          0.14285715, 0., -0., -0.12698413, 0.11111111, 0., -0.0026455, -0.10185185, 0.08333334,
                          0.07692308, 0., 0., -0.07179487, 0.06666667, 0., -0.0005698, -0.06296296, 0.05555556], np.float32).reshape(3, 3, 3)
TRI_UPPER = np.array([4, 5, 6, 0, 2, 3, 0, 0, 1, 10, 11, 12, 0, 8, 9, 0, 0, 7, 16, 17, 18, 0, 14, 15, 0, 0, 13], np.float32).reshape(3, 3, 3)
TRI_UPPER_INV = np.array([0.25, -0.625, 0.375, 0., 0.5, -1.5, 0., 0., 1.,
                          0.1, -0.1375, 0.00535714, 0., 0.125, -0.16071428, 0., 0., 0.14285715,
                          0.0625, -0.07589286, 0.00103022, 0., 0.07142857, -0.08241758, 0., 0., 0.07692308], np.float32).reshape(3, 3, 3)
TRANSPOSED_TRI_LOWER = np.array([1, 2, 4, 0, 3, 5, 0, 0, 6, 7, 8, 10, 0, 9, 11, 0, 0, 12, 13, 14, 16, 0, 15, 17, 0, 0, 18],
                                np.float32).reshape(3, 3, 3)

# ---- test_linalg_block_routines.cpp:207-400: Fill / Get diagonal and sparse blocks, 12 x 12 matrix, 2 x 2 blocks ----
ARANGE_BLOCKS = np.arange(24, dtype=np.float32).reshape(6, 2, 2)
SPARSE_COORDS = np.array([[0, 0], [0, 1], [2, 0], [3, 3], [2, 4], [5, 5]], np.int32)
SPARSE_FILLED = np.zeros((12, 12), np.float32)
SPARSE_FILLED[0:2, 0:4] = [[0, 1, 4, 5], [2, 3, 6, 7]]
SPARSE_FILLED[4:6, 0:2] = [[8, 9], [10, 11]]
SPARSE_FILLED[4:6, 8:10] = [[16, 17], [18, 19]]
SPARSE_FILLED[6:8, 6:8] = [[12, 13], [14, 15]]
SPARSE_FILLED[10:12, 10:12] = [[20, 21], [22, 23]]
TRANSPOSE_FILL_BLOCKS = np.array([4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19], np.float32).reshape(3, 2, 2)
TRANSPOSE_FILL_COORDS = np.array([[0, 1], [2, 0], [2, 4]], np.int32)
SPARSE_FILLED_2 = SPARSE_FILLED.copy()
SPARSE_FILLED_2[0:2, 4:6] = [[8, 10], [9, 11]]
SPARSE_FILLED_2[2:4, 0:2] = [[4, 6], [5, 7]]
SPARSE_FILLED_2[8:10, 4:6] = [[16, 18], [17, 19]]
