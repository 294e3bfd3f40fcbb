// Dev: can a kernel take ~100 KB of dynamic LDS on this device/runtime?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(64) void k(float *o)
{
    extern __shared__ float4 b[];
    b[threadIdx.x * 97] = float4{1, 2, 3, 4};
    __syncthreads();
    o[threadIdx.x] = b[threadIdx.x * 97].y;
}
int main()
{
    int v = 0;
    hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, 0);
    printf("max LDS per block attr: %d\n", v);
    hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, 0);
    printf("opt-in LDS per block attr: %d\n", v);
    float *o;
    (void)hipMalloc(&o, 4096);
    for (int bytes : {65536, 99840, 131072, 163840}) {
        hipError_t e1 = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), bytes, 0, o);
        hipError_t e2 = hipGetLastError();
        hipError_t e3 = hipDeviceSynchronize();
        printf("%6d B: setattr %s, launch %s, sync %s\n", bytes, hipGetErrorString(e1), hipGetErrorString(e2),
               hipGetErrorString(e3));
    }
    return 0;
}
