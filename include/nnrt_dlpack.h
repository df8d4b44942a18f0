/*
 * nnrt_dlpack.h -- DLPack entry points of the MI355X-native DeformableMeshToImageFitter ("tensors via
 * DLPack (DLManagedTensor*) from torch-ROCm or numpy").
 *
 * Each function validates the tensors (device, dtype, shape, compact row-major layout) and forwards to the pointer
 * entry point of nnrt_mi355x.h that it mirrors. Tensors are BORROWED: the caller keeps ownership, the library never calls
 * a deleter and keeps no reference after the call returns. Device tensors must be kDLROCM (or kDLROCMHost for the host
 * arrays noted) on the handle's device; host arrays may be kDLCPU. Errors: NNRT_ERROR_ARGUMENT with a message naming
 * the tensor and the mismatch (reference behaviour: utility::LogError -> RuntimeError).
 *
 * The DLPack structures are the stable DLPack C ABI (v0.6+ layout); when the real dlpack.h is included first
 * (DLPACK_VERSION defined), its definitions are used instead.
 */
#ifndef NNRT_DLPACK_H
#define NNRT_DLPACK_H

#include <stdint.h>

#include "nnrt_mi355x.h"

#ifndef DLPACK_VERSION
typedef enum { kDLCPU = 1, kDLCUDA = 2, kDLCUDAHost = 3, kDLROCM = 10, kDLROCMHost = 11 } DLDeviceType;
typedef struct {
	int32_t device_type;
	int32_t device_id;
} DLDevice;
typedef enum { kDLInt = 0, kDLUInt = 1, kDLFloat = 2, kDLBool = 6 } DLDataTypeCode;
typedef struct {
	uint8_t code;
	uint8_t bits;
	uint16_t lanes;
} DLDataType;
typedef struct {
	void* data;
	DLDevice device;
	int32_t ndim;
	DLDataType dtype;
	int64_t* shape;
	int64_t* strides; /* NULL: compact row-major */
	uint64_t byte_offset;
} DLTensor;
typedef struct DLManagedTensor {
	DLTensor dl_tensor;
	void* manager_ctx;
	void (*deleter)(struct DLManagedTensor* self);
} DLManagedTensor;
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* HierarchicalGraphWarpField(nodes, ...) (cpp/geometry/HierarchicalGraphWarpField.h:37-48, pybind geometry.cpp:278-320):
 * nodes float32 [N,3] on the host (kDLCPU / kDLROCMHost) or on a ROCm device (copied to the host for construction). */
nnrt_status nnrt_warp_field_create_dlpack(const DLManagedTensor* nodes, float node_coverage, int32_t threshold_nodes_by_distance,
                                          int32_t anchor_count, int32_t minimum_valid_anchor_count, int32_t coverage_method,
                                          int32_t layer_count, int32_t max_vertex_degree, const float* h_layer_radii, int32_t device,
                                          nnrt_warp_field** out);

/* DeformableMeshToImageFitter::FitToImage(warp_field, canonical_mesh, reference_image, depth, mask, K, E, scale)
 * (cpp/alignment/DeformableMeshToImageFitter.cpp:278-314) == nnrt_fitter_fit_to_image: vertices / normals float32 [V,3],
 * faces int64 [F,3], depth float32 [H,W], mask bool or uint8 [H,W] (NULL: all valid), all on the warp field's ROCm
 * device; K float64 [3,3] and E float64 [4,4] on the host. */
nnrt_status nnrt_fitter_fit_to_image_dlpack(nnrt_fitter* fitter, nnrt_warp_field* warp_field, const DLManagedTensor* vertices,
                                            const DLManagedTensor* normals, const DLManagedTensor* faces, const DLManagedTensor* depth,
                                            const DLManagedTensor* mask, const DLManagedTensor* K, const DLManagedTensor* E,
                                            float depth_scale, void* stream);

/* nnrt.rendering.rasterize_ndc_triangles (cpp/pybind/rendering/rendering.cpp:36-43) == nnrt_rasterize_ndc_triangles:
 * face_ndc float32 [F,3,3] and clip_mask bool / uint8 [F] (NULL: all faces) in; the caller-allocated fragment tensors
 * pixel_faces int64 [H,W,Kf], depths float32 [H,W,Kf], barycentrics float32 [H,W,Kf,3], distances float32 [H,W,Kf]
 * out (H, W, Kf = faces_per_pixel from pixel_faces' shape). All on one ROCm device (the face_ndc tensor's). */
nnrt_status nnrt_rasterize_ndc_triangles_dlpack(const DLManagedTensor* face_ndc, const DLManagedTensor* clip_mask, float blur_radius_pixels,
                                                int32_t perspective_correct_barycentric_coordinates, int32_t clip_barycentric_coordinates,
                                                int32_t cull_back_faces, const DLManagedTensor* pixel_faces, const DLManagedTensor* depths,
                                                const DLManagedTensor* barycentrics, const DLManagedTensor* distances, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NNRT_DLPACK_H */
