// Probe: fp64 MFMA layout check + fp64 MFMA / VALU FMA throughput on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

// D[16x16] = A[16x4] * B[4x16]; lane l: A[l&15][l>>4], B[l>>4][l&15]; D row=(l>>4)+4r, col=l&15
__global__ void layout(const double* A, const double* B, double* D){
  int l=threadIdx.x;
  double a=A[(l&15)*4+(l>>4)], b=B[(l>>4)*16+(l&15)];
  d4 c={0,0,0,0};
  c=__builtin_amdgcn_mfma_f64_16x16x4f64(a,b,c,0,0,0);
  for(int r=0;r<4;r++) D[((l>>4)+4*r)*16+(l&15)]=c[r];
}
template<int NACC>
__global__ void mfma_rate(double* out, int iters){
  int l=threadIdx.x;
  double a=1.0+l*1e-3, b=1.0-l*1e-3;
  d4 c[NACC];
  for(int i=0;i<NACC;i++) c[i]=(d4){0,0,0,0};
  for(int it=0;it<iters;it++){
#pragma unroll
    for(int i=0;i<NACC;i++) c[i]=__builtin_amdgcn_mfma_f64_16x16x4f64(a,b,c[i],0,0,0);
  }
  double s=0; for(int i=0;i<NACC;i++) s+=c[i][0]+c[i][1]+c[i][2]+c[i][3];
  out[blockIdx.x*blockDim.x+threadIdx.x]=s;
}
__global__ void valu_rate(double* out, int iters){
  int l=threadIdx.x;
  double a=1.0+l*1e-9, b=1.0-l*1e-9;
  double c0=0,c1=0,c2=0,c3=0,c4=0,c5=0,c6=0,c7=0;
  for(int it=0;it<iters;it++){
#pragma unroll
    for(int k=0;k<8;k++){
      c0=fma(a,b,c0);c1=fma(a,c0,c1);c2=fma(b,a,c2);c3=fma(a,c2,c3);
      c4=fma(a,b,c4);c5=fma(b,c4,c5);c6=fma(a,b,c6);c7=fma(b,c6,c7);
    }
  }
  out[blockIdx.x*blockDim.x+threadIdx.x]=c0+c1+c2+c3+c4+c5+c6+c7;
}
int main(){
  // layout
  std::vector<double> A(64),B(64),D(256),R(256);
  for(int i=0;i<16;i++)for(int k=0;k<4;k++)A[i*4+k]=i*10+k+1;
  for(int k=0;k<4;k++)for(int j=0;j<16;j++)B[k*16+j]=(k+1)*100+j*7;
  for(int i=0;i<16;i++)for(int j=0;j<16;j++){double s=0;for(int k=0;k<4;k++)s+=A[i*4+k]*B[k*16+j];R[i*16+j]=s;}
  double *dA,*dB,*dD; CHK(hipMalloc(&dA,512));CHK(hipMalloc(&dB,512));CHK(hipMalloc(&dD,2048));
  CHK(hipMemcpy(dA,A.data(),512,hipMemcpyHostToDevice));CHK(hipMemcpy(dB,B.data(),512,hipMemcpyHostToDevice));
  layout<<<1,64>>>(dA,dB,dD); CHK(hipDeviceSynchronize());
  CHK(hipMemcpy(D.data(),dD,2048,hipMemcpyDeviceToHost));
  int bad=0; for(int i=0;i<256;i++) if(D[i]!=R[i]) bad++;
  printf("layout mismatches: %d\n",bad);
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p,0));
  printf("device %s CUs %d clock %d kHz\n",p.gcnArchName,p.multiProcessorCount,p.clockRate);
  double* out; CHK(hipMalloc(&out,sizeof(double)*1<<24));
  hipEvent_t e0,e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters=4000;
  for(int wpb : {4,8,16}){
    int blocks=256*2; float ms;
    mfma_rate<8><<<blocks,64*wpb>>>(out,10); CHK(hipDeviceSynchronize());
    hipEventRecord(e0); mfma_rate<8><<<blocks,64*wpb>>>(out,iters); hipEventRecord(e1); CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms,e0,e1);
    double fl=2.0*16*16*4*8.0*iters*blocks*wpb;
    printf("MFMA f64 16x16x4, %d waves/WG, %d WGs: %.2f TFLOP/s\n",wpb,blocks,fl/ms/1e9);
    valu_rate<<<blocks,64*wpb>>>(out,10); CHK(hipDeviceSynchronize());
    hipEventRecord(e0); valu_rate<<<blocks,64*wpb>>>(out,iters/8); hipEventRecord(e1); CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms,e0,e1);
    fl=2.0*64*8*8.0*(iters/8)*blocks*wpb;
    printf("VALU f64 fma,       %d waves/WG, %d WGs: %.2f TFLOP/s\n",wpb,blocks,fl/ms/1e9);
  }
  return 0;
}
