// tfusion/cuda/projective_icp.hpp -- cuda::ProjectiveICP (tfusion/include/tfusion/cuda/
// projective_icp.hpp:9-46, tfusion/src/projective_icp.cpp:66-213) for MI355X, header-only over
// the C-ABI of libtfusion_hip.so.
//
// The tracker runs on a context: TopFu::icp() returns the one bound to the TopFu's context (its
// setters change the parameters the TopFu's frames use, as the reference's icp_ object's do);
// a stand-alone ProjectiveICP creates a small context of its own on the first estimateTransform,
// sized to that call's level-0 maps.  estimateTransform copies the caller's pyramids into the
// context and runs the persistent ICP kernel (all levels and iterations in one launch).
#pragma once
#include "../../tfusion_hip.h"
#include "../types.hpp"

#include <stdexcept>
#include <vector>

namespace tfusion
{
    namespace cuda
    {
        class ProjectiveICP
        {
        public:
            enum { MAX_PYRAMID_LEVELS = 4 };

            typedef std::vector<Depth> DepthPyr;
            typedef std::vector<Cloud> PointsPyr;
            typedef std::vector<Normals> NormalsPyr;

            // projective_icp.cpp:68-76: 20 degrees, 0.1 m, iterations {10, 5, 4, 0}
            ProjectiveICP() : angle_thres_(deg2rad(20.f)), dist_thres_(0.1f) { setIterationsNum({ 10, 5, 4, 0 }); }
            virtual ~ProjectiveICP() { if (own_) tf_destroy(own_); }
            ProjectiveICP(const ProjectiveICP&) = delete;
            ProjectiveICP& operator=(const ProjectiveICP&) = delete;

            float getDistThreshold() const { return dist_thres_; }
            void setDistThreshold(float distance) { dist_thres_ = distance; push(); }
            float getAngleThreshold() const { return angle_thres_; }
            void setAngleThreshold(float angle) { angle_thres_ = angle; push(); }

            void setIterationsNum(const std::vector<int>& iters)      // projective_icp.cpp:92-101
            {
                if (iters.size() >= MAX_PYRAMID_LEVELS)
                    iters_.assign(iters.begin(), iters.begin() + MAX_PYRAMID_LEVELS);
                else {
                    iters_ = std::vector<int>(MAX_PYRAMID_LEVELS, 0);
                    std::copy(iters.begin(), iters.end(), iters_.begin());
                }
                push();
            }
            int getUsedLevelsNum() const                               // projective_icp.cpp:103-108
            {
                int i = MAX_PYRAMID_LEVELS - 1;
                for (; i >= 0 && !iters_[i]; --i) {}
                return i + 1;
            }

            // the Frame overload is CV_Assert(!"Not implemented") in the reference (projective_icp.cpp:110-122)
            virtual bool estimateTransform(Affine3f&, const Intr&, const Frame&, const Frame&)
            {
                throw std::logic_error("ProjectiveICP::estimateTransform(Frame): Not implemented");
            }
            // the depth-pyramid variant (projective_icp.cpp:124-166) is not on this path: TopFu
            // tracks with the point pyramids (topfu.cpp:242)
            virtual bool estimateTransform(Affine3f&, const Intr&, const DepthPyr&, const NormalsPyr, const DepthPyr,
                                           const NormalsPyr)
            {
                throw std::logic_error("ProjectiveICP::estimateTransform(depth pyramids): not implemented on MI355X "
                                       "(the point-pyramid overload is the one TopFu uses)");
            }
            // projective_icp.cpp:169-213: affine = Identity, then coarse to fine; false when the
            // normal matrix is singular (|det| < 1e-15 or NaN), affine holding the last composition
            virtual bool estimateTransform(Affine3f& affine, const Intr& intr, const PointsPyr& vcurr, const NormalsPyr ncurr,
                                           const PointsPyr vprev, const NormalsPyr nprev)
            {
                const int levels = getUsedLevelsNum();
                if (levels > 3) throw std::invalid_argument("ProjectiveICP: at most 3 pyramid levels on MI355X");
                if ((int)vcurr.size() < levels || (int)ncurr.size() < levels || (int)vprev.size() < levels ||
                    (int)nprev.size() < levels)
                    throw std::invalid_argument("ProjectiveICP::estimateTransform: pyramid shorter than the used levels");
                tf_ctx* c = worker(vcurr[0].cols(), vcurr[0].rows());
                tf_map_level cl[3], pl[3];
                for (int l = 0; l < levels; ++l) {
                    cl[l].points = vcurr[l].ptr(); cl[l].points_step = vcurr[l].step();
                    cl[l].normals = ncurr[l].ptr(); cl[l].normals_step = ncurr[l].step();
                    pl[l].points = vprev[l].ptr(); pl[l].points_step = vprev[l].step();
                    pl[l].normals = nprev[l].ptr(); pl[l].normals_step = nprev[l].step();
                }
                const float in[4] = { intr.fx, intr.fy, intr.cx, intr.cy };
                float rt[12];
                int ok = 0, iters = 0;
                const tf_status s = tf_icp_estimate(c, in, cl, pl, levels, rt, &ok, &iters);
                if (s != TF_OK) throw std::runtime_error(std::string("tf_icp_estimate: ") + tf_status_string(s));
                affine = affine_from_rt(rt);
                last_iterations_ = iters;
                return ok != 0;
            }

            // MI355X additions: the context TopFu binds its tracker to, and the iteration count
            // of the last estimateTransform
            void bind(tf_ctx* ctx) { bound_ = ctx; push(); }
            int lastIterations() const { return last_iterations_; }

        private:
            void push()
            {
                if (bound_) push_to(bound_);
                else if (own_) push_to(own_);
            }
            tf_ctx* worker(int cols, int rows)
            {
                if (bound_) return bound_;
                tf_params p;
                if (own_) {
                    tf_get_params(own_, &p);
                    if (p.cols == cols && p.rows == rows) return own_;
                    tf_destroy(own_);
                    own_ = nullptr;
                }
                tf_default_params(&p);
                p.cols = cols; p.rows = rows;
                p.n_buckets = 16; p.n_excess = 16; p.n_blocks = 16;      // tracking only: no scene
                p.vis_capacity = 16; p.max_render_blocks = 16;
                const tf_status s = tf_create(&p, &own_);
                if (s != TF_OK) throw std::runtime_error(std::string("ProjectiveICP: tf_create: ") + tf_status_string(s));
                push_to(own_);
                return own_;
            }
            void push_to(tf_ctx* c)
            {
                int it[4] = { iters_[0], iters_[1], iters_[2], iters_[3] };
                const tf_status s = tf_icp_set_params(c, dist_thres_, angle_thres_, it);
                if (s != TF_OK) throw std::invalid_argument(std::string("tf_icp_set_params: ") + tf_status_string(s));
            }

            std::vector<int> iters_;
            float angle_thres_;
            float dist_thres_;
            tf_ctx* bound_ = nullptr;        // TopFu's context (not owned)
            tf_ctx* own_ = nullptr;          // stand-alone context (owned)
            int last_iterations_ = 0;
        };
    }
}
