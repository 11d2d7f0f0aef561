/*
 * rt_image.h -- output/format step of the render path (librt_scene.so, host only).
 *
 * Replaces the reference's display of the accumulation buffer: CLRaytracer::RenderFrame
 * uploads the float4 pixels to a GL_RGBA32F texture (CLRaytracer.cpp:25-26, :64-67) that GL
 * shows clamped to [0, 1].  Here the same buffer is written to an image file instead:
 * 8-bit RGB, v8 = floor(clamp(v, 0, 1) * 255 + 0.5) (NaN -> 0), rows flipped because the
 * kernel's row 0 is the bottom of the picture (kernel_bvh.cl:386-403, GL convention).
 *
 * `px` is W*H float4 (16-byte stride, the BUFFER_OUT layout; the 4th lane is ignored).
 * All functions return 0 or a negative rt_status.h code.
 */
#ifndef RT_IMAGE_H
#define RT_IMAGE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* W*H*3 bytes, top row first. */
int rtiToRGB8(const float* px, unsigned W, unsigned H, unsigned char* out);
/* Binary PPM (P6). */
int rtiWritePPM(const char* path, const float* px, unsigned W, unsigned H);
/* PNG, 8-bit RGB, zlib stream of stored (uncompressed) deflate blocks: no external library. */
int rtiWritePNG(const char* path, const float* px, unsigned W, unsigned H);

/* Checkpoint / resume of a progressive render: the reference's whole render state is
 * its accumulation buffer plus m_FrameCount (CLRaytracer.h:30-37; KernelEntry accumulates in place,
 * kernel_bvh.cl:449-455), so a run of N spp can stop after frame f and go on later from the same
 * bits.  Format: "RTACCUM1", u32 W, u32 H, u32 next frame count, the W*H float4 pixels as stored
 * (16-byte stride, 4th lane included), u64 FNV-1a of everything before it.
 * rtiLoadAccum with px == NULL only reads the header (W, H, next frame); a bad magic, size or
 * checksum is RT_PARSE_ERROR, a W x H that differs from the caller's (px != NULL) RT_INVALID_VALUE. */
int rtiSaveAccum(const char* path, const float* px, unsigned W, unsigned H, unsigned next_frame);
int rtiLoadAccum(const char* path, float* px, unsigned* W, unsigned* H, unsigned* next_frame);

#ifdef __cplusplus
}
#endif

#endif /* RT_IMAGE_H */
