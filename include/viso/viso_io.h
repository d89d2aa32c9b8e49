/* viso_amd — frame source: PNG decoding and KITTI calibration (host only).
 *
 * The reference's frame source reads each frame with
 * cv::imread("<location><n>.png", 0) (include/frame_sequence.h:28-30;
 * OpenCV 3.x IMREAD_GRAYSCALE through its libpng decoder).  KITTI odometry
 * sequences (the north star's "KITTI-format grey pairs") are
 * sequences/NN/image_0|1/%06d.png plus calib.txt.  These entry points restate
 * that decoding without OpenCV (zlib inflate, PNG filters, Adam7) so the
 * frame source needs no third-party image library:
 *   - 8-bit grey: the bytes as stored; 1/2/4-bit grey expanded to 0..255
 *     (libpng png_set_expand_gray_1_2_4_to_8); 16-bit grey: the high byte
 *     (png_set_strip_16);
 *   - RGB / RGBA (8- or 16-bit; 16-bit samples to their high byte,
 *     png_set_strip_16) / palette: alpha dropped (png_set_strip_alpha),
 *     palette expanded, then libpng 1.6's png_set_rgb_to_gray(.., 0.299,
 *     0.587) without gamma tables: grey = r if r == g == b, else
 *     (9797 r + 19234 g + 3737 b) >> 15 (truncating; libpng's fixed-point
 *     weights 0.299 * 32768 and 0.587 * 32768 rounded down, blue the rest);
 *   - ancillary chunks are not interpreted (gAMA / sRGB / iCCP: imread sets
 *     no gamma transform; tRNS: expanded to alpha, then stripped); a CRC
 *     error in an ancillary chunk skips the chunk (libpng's default), in a
 *     critical chunk it fails the decode (VISO_ERR_ARG).
 * Parity of the colour conversion against OpenCV itself is unpinned (neither
 * OpenCV nor libpng is in the image); grey PNGs (KITTI) are exact.
 */
#ifndef VISO_IO_H
#define VISO_IO_H

#include <stddef.h>
#include <stdint.h>

#include "viso_c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Width and height of a PNG file (VISO_ERR_ARG if unreadable / not a PNG). */
int viso_png_info(const char* path, int32_t* width, int32_t* height);

/* cv::imread(path, IMREAD_GRAYSCALE) for PNG: width * height grey bytes,
 * continuous rows, into out (cap bytes; VISO_ERR_CAPACITY if too small, with
 * *width / *height set). */
int viso_png_read_grey(const char* path, uint8_t* out, size_t cap, int32_t* width, int32_t* height);

/* The same from a PNG byte stream in memory. */
int viso_png_decode_grey(const uint8_t* data, size_t size, uint8_t* out, size_t cap, int32_t* width,
                         int32_t* height);

/* KITTI odometry calib.txt: left camera P0 -> fx, fy, cx, cy; stereo
 * baseline = -P1[0][3] / P1[0][0] (metres). */
int viso_kitti_calib(const char* path, double* fx, double* fy, double* cx, double* cy, double* baseline);

#ifdef __cplusplus
}
#endif
#endif /* VISO_IO_H */
