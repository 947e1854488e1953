// world_bvh.h — host-side build of the world BVH (DevWorldNode) over a scene's object list.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "device_types.h"
#include "../../include/yart.h"

namespace yart_dev {

struct BuiltWorld {
  std::vector<DevWorldNode> nodes;  // the binary tree, root = nodes[0]
  std::vector<DevWorldNode4> nodes4;  // the 4-wide tree the device walks, root = nodes4[0]
  uint32_t depth4 = 0;              // its inner levels on the deepest root-to-leaf path
  std::vector<uint32_t> objs;       // leaf slots -> object index
  std::vector<double> sph;          // per leaf slot: centre xyz, radius of a plain sphere (else 0)
  uint32_t depth = 0;               // inner levels on the deepest root-to-leaf path
  // The directions in the x-z plane along which a ray lies in a RotateY'd rect's or box's own plane
  // (a local x or z direction component of exactly 0), as sorted "diamond angles" mod pi (kernels.hip
  // plane_diamond), padded with +inf to a power of two. Such a ray can get the reference's t = 0/0 =
  // NaN "hit" outside any box (aarect.rs:111-146, under hittable.rs:217-251); world_closest_bvh
  // sends every ray within kPlaneDirWindow of one of them to the list walk.
  std::vector<double> plane_dirs;
};


// World-space bounds of one list entry: the primitive's own box (sphere ± |r|, rect extent with
// its plane coordinate, box corners, triangle vertices) carried through its wrappers innermost
// first as hit_record undoes them (RotateY's back rotation on the 8 corners, Translate's offset).
// false for kinds that have no box here (meshes: those scenes keep the linear walk).
bool world_bounds(const DevObject& o, double lo[3], double hi[3]);

// Surface-area-heuristic splits (sah, the default; leaves of up to 4 objects), or median splits on
// the centroid's widest axis down to <= 2 objects per leaf; boxes are padded by 1e-7 of their
// magnitude and rounded outward to f32. Any tree gives the linear scan's answer (the walk keeps
// min t, ties to the later object: kernels.hip world_closest_bvh). false if some object has no box.
bool build_world_bvh(const std::vector<DevObject>& objs, BuiltWorld& out, bool sah = true);

// The 4-wide tree's structure: every object in exactly one leaf reachable from the root, every
// child box holding the world box of each object below it, sphere leaves holding plain spheres,
// empty slots without a box, at least two children per node, depth4 the tree's and within the
// walk's 32-slot stack. false with a reason in err.
bool check_world4(const std::vector<DevObject>& objs, const BuiltWorld& w, std::string& err);

}  // namespace yart_dev
