/*
 * asan_main.c -- TEST INFRASTRUCTURE: drives the CPU oracle (tf_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_oracle.py builds it with
 * -fsanitize=address,undefined and runs it).  Frames come from a raw uint16 file the test
 * writes (synthetic orbit); the run covers TopFu::operator() over the sequence (frame 0,
 * tracking, ICP-failure resets), the five RenderImage types, and a swapping + colour pass
 * on small capacities so eviction and capacity exhaustion paths run.
 *
 *   asan_main FRAMES.raw W H N
 */
#include "tf_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int run(const uint16_t* frames, int W, int H, int n, int swapping, int rgb)
{
    tfo_params p;
    tfo_default_params(&p);
    p.cols = W; p.rows = H;
    const float s = (float)W / 640.0f;
    p.fx *= s; p.fy *= s; p.cx *= s; p.cy *= s;
    if (swapping || rgb) {          /* small capacities: saturation, excess chains, eviction */
        p.n_buckets = 0x2000; p.n_excess = 0x800; p.n_blocks = 1024; p.vis_capacity = 0x4000;
        p.voxelSize = 0.01f;
    }
    p.use_swapping = swapping;
    p.swap_transfer_blocks = 64;
    p.voxel_rgb = rgb;
    tfo_ctx* c = tfo_create(&p);
    tfo_ctx* d = tfo_create(&p);
    uint8_t* img = (uint8_t*)malloc((size_t)W * H * 4);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        img[4 * i] = (uint8_t)(i * 7); img[4 * i + 1] = (uint8_t)(i >> 3); img[4 * i + 2] = (uint8_t)(i * 13);
        img[4 * i + 3] = 255;
    }
    int ok = 0;
    for (int k = 0; k < n; ++k) {
        const uint16_t* f = frames + (size_t)k * W * H;
        ok += rgb ? tfo_process_frame_rgb(c, f, img, 0) : tfo_process_frame(c, f);
        if (k == n / 2 && tfo_copy_state(d, c) != 0) { fprintf(stderr, "copy_state failed\n"); return 1; }
    }
    for (int t = 0; t <= 4; ++t) tfo_render_image_type(c, t);
    tfo_render_image(c, img);
    tfo_counters cn;
    tfo_get_counters(c, &cn);
    printf("swapping %d rgb %d frames %d ok %d resets %d visible %d free %d\n", swapping, rgb, n, ok, cn.n_resets,
           cn.noVisibleEntries, cn.lastFreeBlockId);
    free(img);
    tfo_destroy(c);
    tfo_destroy(d);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 5) { fprintf(stderr, "usage: %s FRAMES.raw W H N\n", argv[0]); return 2; }
    const int W = atoi(argv[2]), H = atoi(argv[3]), n = atoi(argv[4]);
    const size_t bytes = (size_t)W * H * n * sizeof(uint16_t);
    uint16_t* frames = (uint16_t*)malloc(bytes);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(frames, 1, bytes, f) != bytes) { fprintf(stderr, "cannot read %s\n", argv[1]); return 2; }
    fclose(f);
    int r = run(frames, W, H, n, 0, 0);
    if (!r) r = run(frames, W, H, n, 1, 0);
    if (!r) r = run(frames, W, H, n, 0, 1);
    free(frames);
    if (!r) printf("ASAN_MAIN_DONE\n");
    return r;
}
