/*
 * lit_model.c -- CPU statistics for the free-literal path: visited
 * positions of the reference parse whose slot has no earlier position in the
 * window (literals whatever the inserted set), per workload.  Design aid only.
 *   gcc -O2 -I gibson_amd/csrc tools/lit_model.c -o /tmp/lit_model && /tmp/lit_model KIND N COUNT
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "synth.h"
static inline uint32_t slot(const uint8_t *b, uint32_t p){uint32_t hi=((uint32_t)b[p]<<8)|b[p+1],lo=((uint32_t)b[p+1]<<8)|b[p+2];return (hi-5u*lo)&0xFFFFu;}
int main(int argc,char**argv){int kind=atoi(argv[1]);uint32_t n=atoi(argv[2]),count=atoi(argv[3]);
 uint8_t*b=malloc(n+64);int32_t*last=malloc(65536*4),*tab=malloc(65536*4);
 uint64_t steps=0,lits=0,free_l=0,runs=0,fl_same16=0;
 for(uint32_t v=0;v<count;v++){syn_generate(kind,0x5EED0002ull+kind,v,b,n);
  for(int i=0;i<65536;i++){last[i]=-1;tab[i]=-1;}
  /* q1 of every position: latest earlier same-slot position */
  int32_t*q1=malloc(n*4);for(uint32_t p=0;p+2<n;p++){uint32_t s=slot(b,p);q1[p]=last[s];last[s]=p;}
  uint32_t p=0;int prev_free=0;
  while(p+2<n){steps++;uint32_t s=slot(b,p);int32_t r=tab[s];tab[s]=p;
   int fr=!(q1[p]>0 && p-q1[p]-1<8192);
   uint32_t len=0;
   if(r>0&&p-r-1<8192&&p+4<n&&b[r]==b[p]&&b[r+1]==b[p+1]&&b[r+2]==b[p+2]){uint32_t maxlen=n-p-2;if(maxlen>264)maxlen=264;len=3;while(len<maxlen&&b[r+len]==b[p+len])len++;}
   if(len){p+=len;if(p>=n-2)break;tab[slot(b,p-2)]=p-2;tab[slot(b,p-1)]=p-1;prev_free=0;}
   else{lits++;if(fr){free_l++;if(prev_free&&(p&15)!=0)fl_same16++;else runs++;}prev_free=fr;p++;}
  }
  free(q1);}
 printf("kind %d n %u: steps/value %.1f literals %.1f free literals %.1f (%.0f%% of steps); free literals following a free literal in the same 16-block %.1f\n",kind,n,(double)steps/count,(double)lits/count,(double)free_l/count,100.0*free_l/steps,(double)fl_same16/count);}
