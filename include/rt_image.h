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

#ifdef __cplusplus
}
#endif

#endif /* RT_IMAGE_H */
