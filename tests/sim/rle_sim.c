/*
 * rle_sim.c - prefix doubling on the run-length encoded string instead of the bytes: how much
 * list work it would leave. Test infrastructure / measurement aid: the CPU
 * oracle's suffix array (oracle/liboracle.so) filtered to run starts is checked to be the order of
 * the run symbols' strings (byte, type = next run's byte above it, length: ascending for type 0,
 * descending for type 1), then the doubling rounds on that string are replayed.
 *
 *   gcc -O2 -o /tmp/rle_sim tests/sim/rle_sim.c -Loracle -loracle -Ltools -ldatagen \
 *       -Wl,-rpath,$PWD/oracle:$PWD/tools
 *   /tmp/rle_sim 16777216 1      # 1: mixed surrogate, 0: text
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
int oracle_suffix_array(const uint8_t *T, int32_t *SA, int32_t n);
void datagen_mixed(uint8_t *out, size_t n, uint64_t seed);
void datagen_text(uint8_t *out, size_t n, uint64_t seed);
static int cmpu(const void*a,const void*b){uint64_t x=*(uint64_t*)a,y=*(uint64_t*)b;return x<y?-1:x>y;}
int main(int argc,char**argv){
  size_t N=atol(argv[1]); int kind=atoi(argv[2]); uint8_t*T=calloc(N+64,1);
  if(kind) datagen_mixed(T,N,1); else datagen_text(T,N,1);
  int32_t n=(int32_t)(N-8);
  int32_t*SA=malloc(4*(size_t)n); oracle_suffix_array(T,SA,n);
  // runs
  int32_t *rid=malloc(4*(size_t)n); int32_t m=0; int32_t *rs=malloc(4*(size_t)n),*rl=malloc(4*(size_t)n);
  for(int32_t i=0;i<n;i++){ if(i==0||T[i]!=T[i-1]){rs[m]=i;rl[m]=0;m++;} rl[m-1]++; rid[i]=m-1; }
  uint64_t*sym=malloc(8*(size_t)m);
  for(int32_t k=0;k<m;k++){ int up = k+1<m && T[rs[k+1]]>T[rs[k]]; uint64_t L=rl[k]; sym[k]=((uint64_t)T[rs[k]]<<33)|((uint64_t)up<<32)|(up?(0xffffffffu-L):L); }
  uint64_t*srt=malloc(8*(size_t)m); memcpy(srt,sym,8*(size_t)m); qsort(srt,m,8,cmpu);
  int32_t D=0; for(int32_t k=0;k<m;k++) if(k==0||srt[k]!=srt[k-1]) srt[D++]=srt[k];
  // dense rank
  uint32_t*U=malloc(4*((size_t)m+1)); for(int32_t k=0;k<m;k++){ int32_t lo=0,hi=D-1; while(lo<hi){int32_t mid=(lo+hi)/2; if(srt[mid]<sym[k]) lo=mid+1; else hi=mid;} U[k]=lo+1;} U[m]=0;
  int bits=0; while((1u<<bits)<=(uint32_t)D) bits++; int kk=64/bits;
  // SA_R: run starts in byte-SA order
  int32_t*SAR=malloc(4*(size_t)m),*RR=malloc(4*(size_t)m); int32_t r=0;
  for(int32_t q=0;q<n;q++){int32_t i=SA[q]; if(i==0||T[i]!=T[i-1]) SAR[r++]=rid[i];}
  if(r!=m){printf("mismatch %d %d\n",r,m);return 1;}
  // verify SA_R is sorted by U lexicographically (check adjacent)
  long bad=0; for(int32_t q=1;q<m;q++){ int32_t a=SAR[q-1],b=SAR[q]; while(a<m&&b<m&&U[a]==U[b]){a++;b++;} uint32_t x=a<m?U[a]:0,y=b<m?U[b]:0; if(!(x<y)) bad++; }
  printf("n %d runs m %d (%.3f) distinct symbols %d bits %d per key %d; SA_R order violations %ld\n",n,m,(double)m/n,D,bits,kk,bad);
  for(int32_t q=0;q<m;q++) RR[SAR[q]]=q;
  int32_t*LR=malloc(4*((size_t)m+1)),*MR=malloc(4*(size_t)m); int32_t h=0; LR[0]=0;
  for(int32_t k=0;k<m;k++){ if(RR[k]>0){int32_t j=SAR[RR[k]-1]; while(k+h<m&&j+h<m&&U[k+h]==U[j+h]) h++; LR[RR[k]]=h; if(h>0)h--;} else h=0; }
  LR[m]=0; for(int32_t q=0;q<m;q++){int32_t a=LR[q],b=q+1<m?LR[q+1]:0; MR[SAR[q]]=a>b?a:b;}
  long tot=m; for(int t=1;t<20;t++){ long d=(long)kk<<(t-1); long c=0; for(int32_t k=0;k<m;k++) if(MR[k]>=d) c++; if(!c)break; tot+=c; printf("rle round %d depth %ld symbols: list %ld\n",t,d,c);}
  printf("sum of lists (incl round 0) %ld\n",tot);
  return 0;
}
