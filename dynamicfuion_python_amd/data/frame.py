"""Frame / frame-pair / frame-sequence datasets over the DeepDeform directory layout (reference data/frame.py,
data/frame_pair.py, data/frame_sequence.py).

Layout of one sequence (DeepDeform + DeepDeformGraph, e.g. `<base>/test/seq017`)::

    color/000300.jpg  depth/000300.png (uint16, mm)  mask/000000_<segment>.png  intrinsics.txt (4x4 text)
    graph_nodes|graph_edges|graph_edges_weights|graph_clusters|graph_node_deformations/<graph>.bin
    pixel_anchors|pixel_weights/<graph>.bin
    <graph> = <hash>_<segment>_<source:06d>_<target:06d>_geodesic_0.05

Differences from the reference, all deliberate:
* the DEEP_DEFORM base directory is an argument (`base_directory=`) or `$DEEPDEFORM_BASE_DIR` instead of the settings
  singleton (settings/path.py); LOCAL resolves to an `example_data` directory given the same way;
* the colour directory is `color/` when present; the reference joins `line_color/` (data/frame.py:188), a name no
  DeepDeform sequence (nor its own example_data) uses (quirk D2);
* `get_current_frame_graph_warp_field` builds this package's `GraphWarpField` on the GPU from the loaded nodes.
"""
from __future__ import annotations

import enum
import os
import re
import typing

import numpy as np

from . import io as dio


class DataSplit(enum.Enum):
    TEST = "test"
    VALIDATION = "val"
    TRAIN = "train"


class DatasetType(enum.Enum):
    DEEP_DEFORM = 0
    LOCAL = 1
    CUSTOM = 2


def make_frame_file_name_mask(name: str, extension: str) -> str:
    """'frame-000042.color', '.png' -> 'frame-{:06d}.color.png': the first digit run becomes a zero-padded field
    (data/frame.py:24-36)."""
    m = re.search(r"\d+", name)
    if m is None:
        raise ValueError(f"frame file name '{name}' holds no frame index")
    return f"{name[:m.start()]}{{:0{m.end() - m.start()}d}}{name[m.end():]}{extension}"


_NOT_LOADED = "Before a dataset can be used, it has to be loaded with the .load() method."


def _require_loaded(fn):
    def wrapper(self, *a, **k):
        if not self._loaded:
            raise ValueError(_NOT_LOADED)
        return fn(self, *a, **k)
    wrapper.__name__ = fn.__name__
    wrapper.__doc__ = fn.__doc__
    return wrapper


def _find_masked(directory: str, subfolders, extensions, name_test) -> typing.Optional[str]:
    """First file in directory/<subfolder> whose extension matches and whose name passes name_test -> filename mask."""
    for sub in subfolders:
        d = os.path.join(directory, sub)
        if not os.path.isdir(d):
            continue
        for filename in sorted(os.listdir(d)):
            stem, ext = os.path.splitext(filename)
            if ext in extensions and name_test(stem):
                return os.path.join(d, make_frame_file_name_mask(stem, ext))
    return None


class GenericDataset:
    """Resolves the directories and file-name masks of one sequence (data/frame.py:39-236)."""

    def __init__(self, sequence_id: typing.Optional[int] = None, split: typing.Optional[DataSplit] = None,
                 base_dataset_type: DatasetType = DatasetType.DEEP_DEFORM, has_masks: bool = False,
                 custom_frame_directory: typing.Optional[str] = None, masks_subfolder: typing.Optional[str] = None,
                 far_clipping_distance: float = 3.0, mask_lower_threshold: int = 250,
                 base_directory: typing.Optional[str] = None):
        self.sequence_id = sequence_id
        self.split = split
        self._base_dataset_type = base_dataset_type
        self._has_masks = has_masks
        self._custom_frame_directory = custom_frame_directory
        self._masks_subfolder = masks_subfolder
        self.far_clipping_distance = far_clipping_distance
        self.mask_lower_threshold = mask_lower_threshold
        self._base_directory_override = base_directory
        self._loaded = False
        self._sequence_directory = self._color_frame_directory = self._depth_frame_directory = None
        self._color_image_filename_mask = self._depth_image_filename_mask = None
        self._mask_frame_directory = self._mask_image_filename_mask = None
        self._intrinsics_file_path = None

    # -- resolution ---------------------------------------------------------------------------------------------
    def _base_directory(self) -> str:
        if self._base_dataset_type == DatasetType.CUSTOM:
            base = self._custom_frame_directory
            what = "custom_frame_directory"
        else:
            base = self._base_directory_override or os.environ.get(
                "DEEPDEFORM_BASE_DIR" if self._base_dataset_type == DatasetType.DEEP_DEFORM else "DEEPDEFORM_EXAMPLE_DIR",
                None if self._base_dataset_type == DatasetType.DEEP_DEFORM else "example_data")
            what = "base_directory (or $DEEPDEFORM_BASE_DIR)"
        if base is None:
            raise ValueError(f"{self._base_dataset_type.name} datasets need {what} to point at the frame data")
        return base

    def _load_custom(self, base: str):
        self._sequence_directory = self._color_frame_directory = self._depth_frame_directory = base
        if self._has_masks:
            self._mask_frame_directory = base
        # file names at the root first (data/frame.py:104-142), then conventional subfolders (:144-175)
        for filename in sorted(os.listdir(base)):
            stem, ext = os.path.splitext(filename)
            if self._color_image_filename_mask is None and ext in (".png", ".jpg", ".jpeg") and ("line_color" in stem or "rgb" in stem):
                self._color_image_filename_mask = os.path.join(base, make_frame_file_name_mask(stem, ext))
            elif self._depth_image_filename_mask is None and ext == ".png" and "depth" in stem:
                self._depth_image_filename_mask = os.path.join(base, make_frame_file_name_mask(stem, ext))
            elif self._has_masks and self._mask_image_filename_mask is None and ext == ".png" and "mask" in stem:
                self._mask_image_filename_mask = os.path.join(base, make_frame_file_name_mask(stem, ext))
            elif self._intrinsics_file_path is None and ext == ".txt" and "ntrinsics" in stem:
                self._intrinsics_file_path = os.path.join(base, filename)
        four_digits = re.compile(r"\d{4}").match
        if self._depth_image_filename_mask is None:
            self._depth_image_filename_mask = _find_masked(base, ["depth", "depth_images", "depth_frames"], [".png"], four_digits)
            if self._depth_image_filename_mask is None:
                raise ValueError(f"Could not find any depth frame data in {base}")
        if self._color_image_filename_mask is None:
            self._color_image_filename_mask = _find_masked(base, ["color", "line_color", "color_images", "color_frames"],
                                                           [".jpg", ".png"], four_digits)
            if self._color_image_filename_mask is None:
                raise ValueError(f"Could not find any color frame data in {base}")
        if self._has_masks and self._mask_image_filename_mask is None:
            subs = [self._masks_subfolder] if self._masks_subfolder else ["mask", "masks", "mask_images", "omask"]
            self._mask_image_filename_mask = _find_masked(base, subs, [".png"], four_digits)
            if self._mask_image_filename_mask is None:
                raise ValueError(f"Could not find any mask frame data in {base}")

    def _load_deep_deform(self, base: str):
        if self.sequence_id is None or self.split is None:
            raise ValueError(f"A dataset of type {self._base_dataset_type.name} requires an integer sequence_id and a DataSplit; "
                             f"got sequence id {self.sequence_id} and split {self.split}.")
        seq = os.path.join(base, f"{self.split.value}/seq{self.sequence_id:03d}")
        self._sequence_directory = seq
        color = os.path.join(seq, "color")
        self._color_frame_directory = color if os.path.isdir(color) else os.path.join(seq, "line_color")
        self._depth_frame_directory = os.path.join(seq, "depth")
        self._color_image_filename_mask = os.path.join(self._color_frame_directory, "{:06d}.jpg")
        self._depth_image_filename_mask = os.path.join(self._depth_frame_directory, "{:06d}.png")
        if self._has_masks:
            self._mask_frame_directory = os.path.join(seq, self._masks_subfolder or "mask")
            first = sorted(os.listdir(self._mask_frame_directory))[0]
            self._mask_image_filename_mask = os.path.join(self._mask_frame_directory, make_frame_file_name_mask(*os.path.splitext(first)))
        self._intrinsics_file_path = os.path.join(seq, "intrinsics.txt")

    def load(self):
        base = self._base_directory()
        self._mask_image_filename_mask = self._mask_frame_directory = None
        if self._base_dataset_type == DatasetType.CUSTOM:
            self._load_custom(base)
        else:
            self._load_deep_deform(base)
        self._loaded = True
        return self

    # -- accessors ----------------------------------------------------------------------------------------------
    @_require_loaded
    def get_sequence_directory(self) -> str:
        return self._sequence_directory

    @_require_loaded
    def get_color_frame_directory(self) -> str:
        return self._color_frame_directory

    @_require_loaded
    def get_depth_frame_directory(self) -> str:
        return self._depth_frame_directory

    @_require_loaded
    def get_mask_frame_directory(self) -> str:
        return self._mask_frame_directory

    @_require_loaded
    def has_masks(self) -> bool:
        return self._mask_image_filename_mask is not None

    @_require_loaded
    def get_intrinsics_path(self) -> str:
        return self._intrinsics_file_path

    @property
    def far_clipping_distance_mm(self) -> int:
        return int(self.far_clipping_distance * 1000)

    # -- graph data (data/deform_dataset.py:213-266) ---------------------------------------------------------------
    def _graph_path(self, kind: str, graph_filename: str) -> str:
        return os.path.join(self._sequence_directory, kind, graph_filename + ".bin")

    @_require_loaded
    def load_graph_data(self, graph_filename: str, load_deformations: bool = False):
        """(nodes [N,3] f32, edges [N,K] i32, edge weights [N,K] f32, deformations [N,3] or None, clusters [N,1] i32)
        (DeformDataset.load_graph_data, data/deform_dataset.py:233-266)."""
        nodes = dio.load_graph_nodes_or_deformations(self._graph_path("graph_nodes", graph_filename))
        edges = dio.load_graph_edges(self._graph_path("graph_edges", graph_filename))
        weights = dio.load_graph_edges_weights(self._graph_path("graph_edges_weights", graph_filename))
        deformations = dio.load_graph_nodes_or_deformations(self._graph_path("graph_node_deformations", graph_filename)) \
            if load_deformations else None
        clusters = dio.load_graph_clusters(self._graph_path("graph_clusters", graph_filename))
        if not np.isfinite(weights).all():
            raise ValueError(f"{graph_filename}: non-finite edge weights")
        if deformations is not None and not np.isfinite(deformations).all():
            raise ValueError(f"{graph_filename}: non-finite node deformations")
        return nodes, edges, weights, deformations, clusters

    @_require_loaded
    def load_anchors_and_weights(self, graph_filename: str, cropper=None):
        """pixel anchors [H,W,K] i32 and weights [H,W,K] f32 (data/deform_dataset.py:212-231)."""
        anchors = dio.load_int_image(self._graph_path("pixel_anchors", graph_filename))
        weights = dio.load_float_image(self._graph_path("pixel_weights", graph_filename))
        if cropper is not None:
            anchors, weights = cropper(anchors), cropper(weights)
        if not np.isfinite(weights).all():
            raise ValueError(f"{graph_filename}: non-finite pixel weights")
        return anchors, weights

    @_require_loaded
    def graph_filenames(self) -> typing.List[str]:
        d = os.path.join(self._sequence_directory, "graph_edges")
        return sorted(os.path.splitext(f)[0] for f in os.listdir(d)) if os.path.isdir(d) else []


class FrameDataset:
    """Image accessors shared by all frame kinds (data/frame.py:239-268)."""

    def get_color_image_path(self) -> str:
        raise NotImplementedError

    def get_depth_image_path(self) -> str:
        raise NotImplementedError

    def get_mask_image_path(self) -> str:
        raise NotImplementedError

    def load_color_image_numpy(self) -> np.ndarray:
        """BGR, as cv2.imread in the reference."""
        return dio.load_color_image(self.get_color_image_path())[..., ::-1].copy()

    def load_color_image_rgb(self) -> np.ndarray:
        """RGB, as o3d.io.read_image in the fusion app."""
        return dio.load_color_image(self.get_color_image_path())

    def load_depth_image_numpy(self) -> np.ndarray:
        return dio.load_depth_image(self.get_depth_image_path())

    def load_mask_image_numpy(self) -> np.ndarray:
        return dio.load_mask_image(self.get_mask_image_path())


class StandaloneFrameDataset(FrameDataset, GenericDataset):
    """data/frame.py:271-318"""

    def __init__(self, frame_index: int, sequence_id=None, split=None, base_dataset_type=DatasetType.DEEP_DEFORM,
                 has_masks=False, custom_frame_directory=None, masks_subfolder=None, far_clipping_distance=3.0,
                 mask_lower_threshold=250, base_directory=None):
        GenericDataset.__init__(self, sequence_id, split, base_dataset_type, has_masks, custom_frame_directory, masks_subfolder,
                                far_clipping_distance, mask_lower_threshold, base_directory)
        self.frame_index = frame_index

    @_require_loaded
    def get_color_image_path(self) -> str:
        return self._color_image_filename_mask.format(self.frame_index)

    @_require_loaded
    def get_depth_image_path(self) -> str:
        return self._depth_image_filename_mask.format(self.frame_index)

    @_require_loaded
    def get_mask_image_path(self) -> str:
        if not self._has_masks:
            raise ValueError("Trying to retrieve mask path, but the current dataset is defined to have no masks!")
        return self._mask_image_filename_mask.format(self.frame_index)


class SequenceFrameDataset(FrameDataset):
    """One frame of a sequence: explicit paths (data/frame.py:321-338)."""

    def __init__(self, frame_index: int, color_frame_path: str, depth_frame_path: str, mask_frame_path: typing.Optional[str] = None):
        self.frame_index = frame_index
        self.color_image_path = color_frame_path
        self.depth_image_path = depth_frame_path
        self.mask_image_path = mask_frame_path

    def get_color_image_path(self) -> str:
        return self.color_image_path

    def get_depth_image_path(self) -> str:
        return self.depth_image_path

    def get_mask_image_path(self) -> str:
        if self.mask_image_path is None:
            raise ValueError("Trying to retrieve mask path, but the current dataset is defined to have no masks!")
        return self.mask_image_path


def _segment_of(graph_filename: str) -> str:
    return graph_filename.split("_")[1]


class FramePairDataset(GenericDataset):
    """Source/target frame pair with the DeepDeformGraph graph between them (data/frame_pair.py:7-86)."""

    def __init__(self, source_frame_index: int, target_frame_index: int, sequence_id=None, split=None,
                 base_dataset_type=DatasetType.DEEP_DEFORM, has_masks=False, segment_name=None, custom_frame_directory=None,
                 masks_subfolder=None, base_directory=None):
        super().__init__(sequence_id, split, base_dataset_type, has_masks, custom_frame_directory, masks_subfolder,
                         base_directory=base_directory)
        self.graph_filename = None
        self.source_frame_index = source_frame_index
        self.target_frame_index = target_frame_index
        self.segment_name = segment_name

    def load(self):
        super().load()
        if self._base_dataset_type != DatasetType.CUSTOM:
            names = self.graph_filenames()
            if not names:
                raise ValueError(f"no graph data under {self._sequence_directory}/graph_edges")
            first = names[0]
            if self.segment_name is None:
                self.segment_name = _segment_of(first)
            if self._has_masks:
                self._mask_image_filename_mask = os.path.join(self._mask_frame_directory, "{:06d}_" + self.segment_name + ".png")
            self.graph_filename = (f"{first.split('_')[0]}_{self.segment_name}_{self.source_frame_index:06d}_"
                                   f"{self.target_frame_index:06d}_geodesic_0.05")
        return self

    def _frame(self, index: int) -> SequenceFrameDataset:
        if not self._loaded:
            raise ValueError(_NOT_LOADED)
        return SequenceFrameDataset(index, self._color_image_filename_mask.format(index), self._depth_image_filename_mask.format(index),
                                    self._mask_image_filename_mask.format(index) if self._has_masks else None)

    @property
    def source(self) -> SequenceFrameDataset:
        return self._frame(self.source_frame_index)

    @property
    def target(self) -> SequenceFrameDataset:
        return self._frame(self.target_frame_index)

    def get_source_color_image_path(self) -> str:
        return self.source.get_color_image_path()

    def get_target_color_image_path(self) -> str:
        return self.target.get_color_image_path()

    def get_source_depth_image_path(self) -> str:
        return self.source.get_depth_image_path()

    def get_target_depth_image_path(self) -> str:
        return self.target.get_depth_image_path()

    def get_source_mask_image_path(self) -> str:
        return self.source.get_mask_image_path()

    def get_target_mask_image_path(self) -> str:
        return self.target.get_mask_image_path()


class FrameSequenceDataset(GenericDataset, typing.Sequence[SequenceFrameDataset]):
    """Iterable frame sequence (data/frame_sequence.py:12-208). `frame_indices=` restricts the sequence to the frames
    that exist (DeepDeform test sequences ship sparse frames, e.g. 300 and 600); otherwise frames are counted from
    `start_frame_index` upward until the first missing depth file, as in the reference (:68-79)."""

    def __init__(self, sequence_id=None, split=None, start_frame_index: int = 0, frame_count: typing.Optional[int] = None,
                 base_dataset_type=DatasetType.DEEP_DEFORM, has_masks=False, segment_name=None, custom_frame_directory=None,
                 masks_subfolder=None, far_clipping_distance: float = 0.0, mask_lower_threshold: int = 250, base_directory=None,
                 frame_indices: typing.Optional[typing.Sequence[int]] = None):
        super().__init__(sequence_id, split, base_dataset_type, has_masks, custom_frame_directory, masks_subfolder,
                         far_clipping_distance, mask_lower_threshold, base_directory)
        self.segment_name = segment_name
        self.start_frame_index = start_frame_index
        self.frame_count = frame_count
        self._frame_indices = None if frame_indices is None else [int(i) for i in frame_indices]
        self._cursor = 0
        self._resolution = None

    def load(self):
        super().load()
        if self._base_dataset_type != DatasetType.CUSTOM:
            names = self.graph_filenames()
            if self.segment_name is None and names:
                self.segment_name = _segment_of(names[0])
            if self._has_masks and self.segment_name is not None:
                with_segment = os.path.join(self._mask_frame_directory, "{:06d}_" + self.segment_name + ".png")
                if os.path.isfile(with_segment.format(0)):
                    self._mask_image_filename_mask = with_segment
        if self._frame_indices is None:
            if self.frame_count is None:
                end = self.start_frame_index
                while os.path.isfile(self._depth_image_filename_mask.format(end)):
                    end += 1
                if end == self.start_frame_index:
                    raise ValueError(f"Specified sequence start, {self.start_frame_index:d}, is greater or equal than "
                                     f"the total count of frames found on disk {end:d}")
                self.frame_count = end - self.start_frame_index
            self._frame_indices = list(range(self.start_frame_index, self.start_frame_index + self.frame_count))
        else:
            self.frame_count = len(self._frame_indices)
            self.start_frame_index = self._frame_indices[0]
        self._cursor = 0
        self._resolution = dio.load_depth_image(self._depth_image_filename_mask.format(self._frame_indices[0])).shape[:2]
        return self

    @_require_loaded
    def get_frame_at(self, linear_index: int) -> SequenceFrameDataset:
        mask = self._mask_image_filename_mask.format(linear_index) if self._has_masks else None
        return SequenceFrameDataset(linear_index, self._color_image_filename_mask.format(linear_index),
                                    self._depth_image_filename_mask.format(linear_index), mask)

    @_require_loaded
    def get_next_frame(self) -> typing.Optional[SequenceFrameDataset]:
        if self._cursor >= len(self._frame_indices):
            return None
        frame = self.get_frame_at(self._frame_indices[self._cursor])
        self._cursor += 1
        return frame

    @_require_loaded
    def advance_to_frame(self, linear_index: int):
        if linear_index not in self._frame_indices:
            raise ValueError(f"Provided linear_index not within frame range {self._frame_indices[0], self._frame_indices[-1] + 1}")
        self._cursor = self._frame_indices.index(linear_index)

    @_require_loaded
    def get_next_frame_index(self) -> int:
        return self._frame_indices[self._cursor] if self._cursor < len(self._frame_indices) else self._frame_indices[-1] + 1

    @_require_loaded
    def has_more_frames(self) -> bool:
        return self._cursor < len(self._frame_indices)

    @_require_loaded
    def rewind(self):
        self._cursor = 0

    @property
    def resolution(self) -> typing.Tuple[int, int]:
        """(height, width)"""
        if not self._loaded:
            raise ValueError(_NOT_LOADED)
        return self._resolution

    @_require_loaded
    def get_current_graph_name(self) -> typing.Optional[str]:
        """Graph whose source frame is the frame most recently returned (data/frame_sequence.py:115-128)."""
        if self._cursor == 0:
            return None
        current = self._frame_indices[self._cursor - 1]
        for name in self.graph_filenames():
            if int(name.split("_")[2]) == current:
                return name
        return None

    def get_current_pixel_anchors_and_weights(self, cropper=None):
        name = self.get_current_graph_name()
        return (None, None) if name is None else self.load_anchors_and_weights(name, cropper)

    def get_current_frame_graph_warp_field(self, device=None, node_coverage: float = 0.05):
        """GraphWarpField over the loaded graph nodes (data/frame_sequence.py:145-168); None for CUSTOM data or when the
        current frame has no graph."""
        if self._base_dataset_type == DatasetType.CUSTOM:
            return None
        name = self.get_current_graph_name()
        if name is None:
            return None
        from ..nnrt import geometry as G
        nodes, _, _, _, _ = self.load_graph_data(name)
        return G.GraphWarpField(nodes, node_coverage=node_coverage, device=device)

    def __len__(self) -> int:
        if not self._loaded:
            raise ValueError(_NOT_LOADED)
        return self.frame_count

    def __getitem__(self, linear_index):
        return self.get_frame_at(linear_index)

    def __iter__(self):
        for i in self._frame_indices:
            yield self.get_frame_at(i)

    def __repr__(self):
        return (f"<{self.__class__.__name__}. Loaded: {self._loaded}. Sequence directory: {self._sequence_directory}. "
                f"Frames: {self._frame_indices}>")


class StaticFrameSequenceDataset(FrameSequenceDataset):
    """Every frame is frame 0 (data/frame_sequence.py:211-220)."""

    def get_frame_at(self, linear_index: int) -> SequenceFrameDataset:
        if not self._loaded:
            raise ValueError(_NOT_LOADED)
        mask = self._mask_image_filename_mask.format(0) if self._has_masks else None
        return SequenceFrameDataset(linear_index, self._color_image_filename_mask.format(0), self._depth_image_filename_mask.format(0), mask)
