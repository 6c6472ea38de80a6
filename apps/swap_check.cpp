// swap_check.cpp -- the swapping side of the engine API (include/tfusion/engines.hpp):
// Scene(params, useSwapping = true) with its GlobalCache, SwappingEngine_CUDA::
// {IntegrateGlobalIntoLocal, SaveToGlobalMemory} after SceneReconstructionEngine_CUDA::
// {AllocateSceneFromDepth, IntegrateIntoScene}, and GlobalCache::{SaveToFile, ReadFromFile}.
// A camera turns in place through a full circle (ground-truth poses) over a VBA too small for
// the room, so blocks must leave for the cache and come back.  Checks the bookkeeping every
// frame (free count + live blocks = capacity; swapped-out entries hold stored data and are
// not active) and that a cache written to a file reads back identically into a second scene.
// Bit-exactness against the oracle is the Python tests' job (tests/test_gpu_swapping.py).
//
//   ./swap_check [cache_file=/tmp/swap_check.bin]
#include <tfusion/engines.hpp>

#include "synth_depth.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace tfusion;

struct HashEntryBytes { short x, y, z; short pad; int offset, ptr; };

int main(int argc, char** argv)
{
    const char* path = argc > 1 ? argv[1] : "/tmp/swap_check.bin";
    const int cols = 320, rows = 240;
    cuda::setDevice(0);
    TopFuParams p = TopFuParams::default_params();
    p.cols = cols; p.rows = rows;
    const double s = cols / 640.0;
    p.intr = Intr(504.261f * s, 503.905f * s, 352.457f * s, 272.202f * s);
    p.n_buckets = 0x8000; p.n_excess = 0x2000; p.n_blocks = 8192;

    Scene<Voxel_s, VoxelBlockHash> scene(p.sceneParams.get(), true, p);
    SceneReconstructionEngine_CUDA<Voxel_s, VoxelBlockHash> sceneEngine;
    SwappingEngine_CUDA<Voxel_s, VoxelBlockHash> swapEngine;
    RenderState_VH renderState(scene.globalCache->noTotalEntries, Vector2i(cols, rows), p.sceneParams->viewFrustum_min,
                               p.sceneParams->viewFrustum_max);
    sceneEngine.ResetScene(&scene);
    const int n_total = scene.globalCache->noTotalEntries;

    int fails = 0, total_in = 0, total_out = 0;
    std::vector<unsigned short> depth;
    cuda::Depth depth_device;
    cuda::Dists dists;
    std::vector<HashEntryBytes> hash(n_total);
    std::vector<unsigned char> state(n_total), flags(n_total);
    for (int k = 0; k <= 12; ++k) {
        const double a = (30.0 * k) * M_PI / 180.0, ca = std::cos(a), sa = std::sin(a);
        const double R[9] = { ca, 0, sa, 0, 1, 0, -sa, 0, ca }, t[3] = { 0.15, -0.15, 0.6 };
        tfusion_apps::render_depth(R, t, cols, rows, p.intr, depth);
        depth_device.upload(depth.data(), (size_t)cols * 2, rows, cols);
        cuda::computeDists(depth_device, dists, p.intr);
        cuda::waitAllDefaultStream();
        Affine3f c2w = Affine3f::Identity();
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) c2w.matrix(r, c) = (float)R[r * 3 + c];
            c2w.matrix(r, 3) = (float)t[r];
        }
        sceneEngine.AllocateSceneFromDepth(&scene, p.intr, c2w.inv(), dists, &renderState);
        sceneEngine.IntegrateIntoScene(&scene, p.intr, c2w.inv(), dists, &renderState);
        swapEngine.IntegrateGlobalIntoLocal(&scene, &renderState);
        swapEngine.SaveToGlobalMemory(&scene, &renderState);
        int counts[3];
        tf_engine_check(tf_swap_counts(scene.context(), counts), "tf_swap_counts");
        total_in += counts[0];
        total_out += counts[1];

        tf_engine_check(tf_download(scene.context(), TF_BUF_HASH, 0, hash.data(), hash.size() * sizeof(HashEntryBytes)),
                        "hash");
        tf_engine_check(tf_download(scene.context(), TF_BUF_SWAP_STATE, 0, state.data(), state.size()), "state");
        tf_engine_check(tf_download(scene.context(), TF_BUF_SWAP_STORED_FLAGS, 0, flags.data(), flags.size()), "flags");
        std::vector<char> used(p.n_blocks, 0);
        int live = 0, bad = 0;
        for (int i = 0; i < n_total; ++i) {
            const int ptr = hash[i].ptr;
            if (ptr >= 0) {
                if (used[ptr]++) ++bad;                                   // a block held twice
                ++live;
            } else if (ptr == -1 && (!flags[i] || state[i] == 2)) ++bad;  // swapped out: stored, not active
        }
        const tf_stats st = scene.counters();
        if (bad || st.lastFreeBlockId + 1 + live != p.n_blocks) {
            ++fails;
            std::printf("MISMATCH frame %d: live %d free %d bad %d\n", k, live, st.lastFreeBlockId + 1, bad);
        }
    }
    if (total_in == 0 || total_out == 0) {
        ++fails;
        std::printf("MISMATCH: no transfer (in %d out %d)\n", total_in, total_out);
    }

    // GlobalCache::SaveToFile / ReadFromFile into a second swapping scene
    scene.globalCache->SaveToFile(path);
    Scene<Voxel_s, VoxelBlockHash> scene2(p.sceneParams.get(), true, p);
    scene2.globalCache->ReadFromFile(path);
    std::remove(path);
    int stored = 0;
    std::vector<Voxel_s> b1(512), b2(512);
    for (int i = 0; i < n_total; ++i) {
        const bool h1 = scene.globalCache->HasStoredData(i), h2 = scene2.globalCache->HasStoredData(i);
        if (h1 != h2) { ++fails; std::printf("MISMATCH: stored flag %d\n", i); break; }
        if (!h1 || stored++ % 97) continue;                               // every 97th stored block
        scene.globalCache->GetStoredVoxelBlock(i, b1.data());
        scene2.globalCache->GetStoredVoxelBlock(i, b2.data());
        if (std::memcmp(b1.data(), b2.data(), 512 * sizeof(Voxel_s))) { ++fails; std::printf("MISMATCH: block %d\n", i); break; }
    }
    std::printf("swap_check frames 13 swapped in %d out %d stored %d: %s\n", total_in, total_out, stored,
                fails ? "MISMATCH" : "MATCH");
    return fails ? 1 : 0;
}
