// ref_pin.cpp -- TEST INFRASTRUCTURE.  Runs the reference's OWN self-contained
// arithmetic (compiled straight from /root/reference/tfusion/include, no stand-in
// headers) on deterministic inputs and writes golden vectors used to pin the CPU
// oracle (oracle/tf_oracle.c).  Built by oracle/Makefile into oracle/_ref/.
//
// Pinned reference pieces:
//   Matrix4<float>::inv                 Matrix.hpp:173-233  (alloc: M_d.inv(invM_d), SceneReconstructionEngine_host.cu:102-103)
//   Matrix4<float> * Vector4<float>     Matrix.hpp:126-133  (every projection on the path)
//   Vector3<float>::toShortFloor        Vector.hpp:228-230  (TO_SHORT_FLOOR3, SceneReconstructionEngine.hpp:246)
//   Vector3<float>::toIntFloor(resid)   Vector.hpp:236-240  (TO_INT_FLOOR3, RepresentationAccess.hpp:141)
//   Vector3<float>::toIntRound / ROUND  Vector.hpp:210-212, MathUtils.hpp:20 (readFromSDF_float_uninterpolated)
//   dot / length (generic)              Vector.hpp:814-824  (castRay totalLength, VisualisationEngine_Shared.hpp:116)
//   Voxel_s layout / conversions        VoxelTypes.hpp:69-92
//   MIN-based TSDF update arithmetic     MathUtils.hpp:3-4 with Voxel_s (SceneReconstructionEngine.hpp:56-68)
//   interpolateBilinear<uchar>          PixelUtils.hpp:8-32 (computeUpdatedVoxelColorInfo's RGB sample,
//                                       SceneReconstructionEngine.hpp:138)
//   colour running average              Vector3f / Vector3u operators, TO_FLOAT3 / TO_UCHAR3 (Math.hpp:56-68,
//                                       Vector.hpp:242-244) with Voxel_s_rgb (SceneReconstructionEngine.hpp:124-147)
//   Voxel_s_rgb layout / initial value   VoxelTypes.hpp:39-67
#include "Math.hpp"
#include "tfusion/cuda/VoxelTypes.hpp"
#include "tfusion/cuda/PixelUtils.hpp"
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <string>

static uint64_t g_state = 0x243F6A8885A308D3ull;
static uint32_t rnd_u32() { g_state ^= g_state << 13; g_state ^= g_state >> 7; g_state ^= g_state << 17; return (uint32_t)(g_state >> 11); }
static float rnd_f(float lo, float hi) { return lo + (hi - lo) * (float)(rnd_u32() & 0xFFFFFF) / 16777216.0f; }

static void write_f32(const std::string& path, const std::vector<float>& v)
{
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); return; }
    fwrite(v.data(), sizeof(float), v.size(), f);
    fclose(f);
}

static void random_rigid(float rt[12])
{   // rotation from a random unit quaternion, translation in [-2,2]
    float q[4]; float n = 0;
    for (int i = 0; i < 4; ++i) { q[i] = rnd_f(-1, 1); n += q[i] * q[i]; }
    n = 1.0f / sqrtf(n);
    for (int i = 0; i < 4; ++i) q[i] *= n;
    float w = q[0], x = q[1], y = q[2], z = q[3];
    float R[9] = { 1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                   2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                   2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y) };
    for (int r = 0; r < 3; ++r) { for (int c = 0; c < 3; ++c) rt[r * 4 + c] = R[r * 3 + c]; rt[r * 4 + 3] = rnd_f(-2, 2); }
}

int main(int argc, char** argv)
{
    std::string out = argc > 1 ? argv[1] : ".";
    // 1. Matrix4f::inv on rigid poses (column-major load exactly as topfu.cpp:246-249) and general matrices
    {
        std::vector<float> io;
        const int N = 256;
        for (int k = 0; k < N; ++k) {
            float m[16];
            if (k < 192) {
                float rt[12]; random_rigid(rt);
                Matrix4f M(rt[0], rt[4], rt[8], 0.f, rt[1], rt[5], rt[9], 0.f, rt[2], rt[6], rt[10], 0.f, rt[3], rt[7], rt[11], 1.f);
                memcpy(m, M.m, sizeof(m));
            } else {
                for (int i = 0; i < 16; ++i) m[i] = rnd_f(-3, 3);
            }
            Matrix4f M(m), Inv;
            bool ok = M.inv(Inv);
            io.insert(io.end(), m, m + 16);
            io.insert(io.end(), Inv.m, Inv.m + 16);
            io.push_back(ok ? 1.f : 0.f);
        }
        write_f32(out + "/ref_pin_inv.bin", io);
    }
    // 2. Matrix4f * Vector4f
    {
        std::vector<float> io;
        for (int k = 0; k < 1024; ++k) {
            float m[16], v[4];
            for (int i = 0; i < 16; ++i) m[i] = rnd_f(-2, 2);
            for (int i = 0; i < 4; ++i) v[i] = rnd_f(-5, 5);
            Matrix4f M(m); Vector4f V(v[0], v[1], v[2], v[3]);
            Vector4f R = M * V;
            io.insert(io.end(), m, m + 16); io.insert(io.end(), v, v + 4);
            io.push_back(R.x); io.push_back(R.y); io.push_back(R.z); io.push_back(R.w);
        }
        write_f32(out + "/ref_pin_m4v.bin", io);
    }
    // 3. floor / round conversions
    {
        std::vector<float> io;
        for (int k = 0; k < 4096; ++k) {
            float p[3];
            for (int i = 0; i < 3; ++i) {
                float base = rnd_f(-300, 300);
                // include exact integers and half-integers (knife edges)
                int sel = rnd_u32() % 4;
                p[i] = sel == 0 ? floorf(base) : (sel == 1 ? floorf(base) + 0.5f : base);
            }
            Vector3f P(p[0], p[1], p[2]);
            Vector3s s = P.toShortFloor();
            Vector3f resid; Vector3i fi = P.toIntFloor(resid);
            Vector3i ri = P.toIntRound();
            io.insert(io.end(), p, p + 3);
            io.push_back((float)s.x); io.push_back((float)s.y); io.push_back((float)s.z);
            io.push_back((float)fi.x); io.push_back((float)fi.y); io.push_back((float)fi.z);
            io.push_back(resid.x); io.push_back(resid.y); io.push_back(resid.z);
            io.push_back((float)ri.x); io.push_back((float)ri.y); io.push_back((float)ri.z);
            io.push_back(tfusion::length(P));
        }
        write_f32(out + "/ref_pin_round.bin", io);
    }
    // 4. Voxel_s layout, initial value, conversions and the MIN-based TSDF update
    {
        std::vector<float> io;
        Voxel_s v0;
        io.push_back((float)sizeof(Voxel_s)); io.push_back((float)v0.sdf); io.push_back((float)v0.w_depth);
        const float mu = 0.02f; const int maxW = 100;
        for (int k = 0; k < 8192; ++k) {
            Voxel_s v;
            v.sdf = (short)((int)(rnd_u32() % 65535) - 32767);
            v.w_depth = (uchar)(rnd_u32() % 101);
            float eta = rnd_f(-mu, 0.2f);
            if (k % 7 == 0) eta = -mu;              // boundary
            float oldF = Voxel_s::valueToFloat(v.sdf); int oldW = v.w_depth;
            float newF = MIN(1.0f, eta / mu); int newW = 1;
            newF = oldW * oldF + newW * newF;
            newW = oldW + newW;
            newF /= newW;
            newW = MIN(newW, maxW);
            short out_sdf = Voxel_s::floatToValue(newF);
            io.push_back((float)v.sdf); io.push_back((float)v.w_depth); io.push_back(eta);
            io.push_back((float)out_sdf); io.push_back((float)newW);
        }
        write_f32(out + "/ref_pin_voxel.bin", io);
    }
    // 5. interpolateBilinear<uchar> over an RGBA8 image (PixelUtils.hpp:8-32), at positions inside
    //    computeUpdatedVoxelColorInfo's window [1, W-2] x [1, H-2], integer coordinates included
    //    (the delta == 0 branches); record: x, y, 4 results (the image is written first)
    {
        const int W = 23, H = 17;
        std::vector<Vector4u> img(W * H);
        std::vector<float> io;
        for (int k = 0; k < W * H; ++k) {
            uint32_t r = rnd_u32();
            img[k] = Vector4u((uchar)(r & 255), (uchar)((r >> 8) & 255), (uchar)((r >> 16) & 255), (uchar)((r >> 24) & 255));
            io.push_back((float)img[k].x); io.push_back((float)img[k].y); io.push_back((float)img[k].z); io.push_back((float)img[k].w);
        }
        const Vector2i sz(W, H);
        for (int k = 0; k < 4096; ++k) {
            float x = rnd_f(1.0f, (float)(W - 2)), y = rnd_f(1.0f, (float)(H - 2));
            const int sel = rnd_u32() % 4;
            if (sel == 0) x = floorf(x);
            if (sel == 1) y = floorf(y);
            if (sel == 2) { x = floorf(x); y = floorf(y); }
            const Vector2f pos(x, y);
            Vector4f r = interpolateBilinear(&img[0], pos, sz);
            io.push_back(x); io.push_back(y);
            io.push_back(r.x); io.push_back(r.y); io.push_back(r.z); io.push_back(r.w);
        }
        write_f32(out + "/ref_pin_bilinear.bin", io);
    }
    // 6. Voxel_s_rgb layout and the colour running average of computeUpdatedVoxelColorInfo
    //    (SceneReconstructionEngine.hpp:124-147) in the reference's own vector types; record:
    //    r, g, b, w_color, sample r, g, b, then r', g', b', w_color'
    {
        std::vector<float> io;
        Voxel_s_rgb v0;
        io.push_back((float)sizeof(Voxel_s_rgb)); io.push_back((float)v0.sdf); io.push_back((float)v0.w_depth);
        io.push_back((float)v0.clr.x); io.push_back((float)v0.clr.y); io.push_back((float)v0.clr.z); io.push_back((float)v0.w_color);
        const uchar maxW = 100;
        for (int k = 0; k < 8192; ++k) {
            Voxel_s_rgb voxel;
            voxel.clr = Vector3u((uchar)(rnd_u32() % 256), (uchar)(rnd_u32() % 256), (uchar)(rnd_u32() % 256));
            voxel.w_color = (uchar)(rnd_u32() % 101);
            // an interpolated sample: a convex combination of four uchar values (PixelUtils.hpp:23-24)
            const Vector4f sample(rnd_f(0.f, 255.f), rnd_f(0.f, 255.f), rnd_f(0.f, 255.f), 0.f);
            io.push_back((float)voxel.clr.x); io.push_back((float)voxel.clr.y); io.push_back((float)voxel.clr.z);
            io.push_back((float)voxel.w_color);
            io.push_back(sample.x); io.push_back(sample.y); io.push_back(sample.z);
            Vector3f rgb_measure, oldC, newC; Vector3u buffV3u;
            float newW, oldW;
            buffV3u = voxel.clr;
            oldW = (float)voxel.w_color;
            oldC = TO_FLOAT3(buffV3u) / 255.0f;
            rgb_measure = TO_VECTOR3(sample) / 255.0f;
            newW = 1;
            newC = oldC * oldW + rgb_measure * newW;
            newW = oldW + newW;
            newC /= newW;
            newW = MIN(newW, maxW);
            voxel.clr = TO_UCHAR3(newC * 255.0f);
            voxel.w_color = (uchar)newW;
            io.push_back((float)voxel.clr.x); io.push_back((float)voxel.clr.y); io.push_back((float)voxel.clr.z);
            io.push_back((float)voxel.w_color);
        }
        write_f32(out + "/ref_pin_colour.bin", io);
    }
    printf("ref_pin: wrote goldens to %s\n", out.c_str());
    return 0;
}
