// Replay probe of the JLN person kernel: person_cl_kernel
// <LPV=4, one row per block, packed fine grid, V <= 16> with the product's
// launch (fvp_person_planes_cl: XCD-aware proposal placement, x-split by the
// launch size) and a MODE that removes one part at a time (fvp_person.hip):
//   0 FULL      the kernel as shipped (sanity: equals fvp_person_planes_cl)
//   1 NOPLANES  no plane reductions, atomics or plane stores
//   2 NOTAPS    zeros instead of the tap loads
//   3 ALL_OOB   every tap offset off-image (range-checked loads)
//   4 SETUP     grid loads + tap setup only
//   5 NO_XZ_ATOMICS  FULL without the xz-plane atomics
//   6 NO_XY_ATOMICS  FULL without the xy-plane atomics
//   7 HALF_XZ_ATOMICS  xz atomics from half the lanes (lane-count vs instruction cost)
//   8 XZ_STORES  plain stores instead of the xz atomics (timing only)
// Test tooling only (tools/person_probe.py); not part of libfvp.
#include "../faster-voxelpose_amd/csrc/fvp_person.hip"

template <int MODE>
static void go(dim3 grid, hipStream_t s, const float *cl, const float *fgrid, const fvp_person_spec &spec,
               const float *props, const int32_t *frame_of, float *planes, float *offset, int P, int V, int J,
               int H, int W, int xsplit, unsigned pix_bytes) {
    hipLaunchKernelGGL((fvp::person_cl_kernel<4, false, false, MODE>), grid, dim3(256), 0, s, cl, fgrid,
                       fvp::PersonCoords{}, props, frame_of, spec, nullptr, planes, offset, P, V, J, J, H, W, 1,
                       xsplit, 1, pix_bytes, xsplit == 1 ? 1 : 0);
}

extern "C" int person_probe(int mode, const float *cl, int cp, const float *fgrid, const fvp_person_spec *spec,
                            const float *props, const int32_t *frame_of, int P, int V, int J, int H, int W,
                            float *planes, float *offset, void *stream) {
    if (V > 16 || J > 16 || cp != 16 || spec->bins[2] > 64) return FVP_ERR_SHAPE;
    hipStream_t s = (hipStream_t)stream;
    const int SX = spec->bins[0], SY = spec->bins[1];
    const int xsplit = fvp::person_xsplit(P, SY);
    const size_t n = (xsplit > 1 ? 3 : 2) * (size_t)P * J * SX * SY;
    if (hipMemsetAsync(planes, 0, n * 4, s) != hipSuccess) return 1;
    const dim3 grid((unsigned)((long long)P * SY * xsplit));
    const unsigned pb = (unsigned)cp * 4u;
    switch (mode) {
        case 0: go<0>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 1: go<1>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 2: go<2>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 3: go<3>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 4: go<4>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 5: go<5>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 6: go<6>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 7: go<7>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        case 8: go<8>(grid, s, cl, fgrid, *spec, props, frame_of, planes, offset, P, V, J, H, W, xsplit, pb); break;
        default: return FVP_ERR_SHAPE;
    }
    return (int)hipGetLastError();
}
