/*
 * wave_balance.c -- how unevenly the values of one wave finish in the
 * one-lane-per-value parse (design aid, not part of the product or tests).
 * Per value: an iteration proxy of lzf_parse_lane_kernel (one per literal or
 * match step, free literals four to an iteration, one per 16-byte extension
 * piece past 8 bytes) under the reference parse (src/lzf_c.c:145-274);
 * per wave of 64 consecutive values: max / mean.
 *
 *   gcc -O2 -I gibson_amd/csrc tools/wave_balance.c -o /tmp/wave_balance
 *   /tmp/wave_balance <kind> <n> <count> <seed>
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "synth.h"
static inline uint32_t slot(const uint8_t *b, uint32_t p){uint32_t hi=((uint32_t)b[p]<<8)|b[p+1],lo=((uint32_t)b[p+1]<<8)|b[p+2];return (hi-5u*lo)&0xFFFFu;}
/* per-value lane-parse iteration proxy: one per match or literal step, free
 * literals (no same-slot candidate in the window) merged 4 per iteration */
int main(int argc,char**argv){int kind=atoi(argv[1]);uint32_t n=atoi(argv[2]),count=atoi(argv[3]);uint64_t seed=strtoull(argv[4],0,0);
 uint8_t*b=malloc(n+64);uint32_t*tab=malloc(65536*4),*last=malloc(65536*4);uint8_t*ins=malloc(n);
 double summax=0,summean=0,sum4max=0,sum4mean=0; uint32_t it[64*4];
 for(uint32_t v0=0;v0<count;v0+=256){
  for(uint32_t k=0;k<256;k++){uint32_t v=v0+k;syn_generate(kind,seed,v,b,n);memset(tab,0xFF,65536*4);memset(last,0xFF,65536*4);memset(ins,0,n);
   uint32_t p=0,iters=0,freerun=0;
   while(p+2<n){uint32_t s=slot(b,p);uint32_t r=tab[s];tab[s]=p;ins[p]=1;
     uint32_t any=last[s]; last[s]=p; (void)any;
     int hit=r!=0xFFFFFFFFu&&(p-r-1u)<8192&&p+4<n&&r>0&&b[r]==b[p]&&b[r+1]==b[p+1]&&b[r+2]==b[p+2];
     int free_=(r==0xFFFFFFFFu||(p-r-1u)>=8192);
     if(!hit){ if(free_){ if(freerun%4==0) iters++; freerun++; } else {iters++;freerun=0;} p++; continue;}
     freerun=0; iters++;
     uint32_t maxlen=n-p-2; if(maxlen>264)maxlen=264; uint32_t lim=maxlen>16&&maxlen<19?19:maxlen,m=3; while(m<lim&&b[r+m]==b[p+m])m++;
     iters += m>8 ? (m-8+15)/16 : 0;
     p+=m; if(p>=n-2)break; tab[slot(b,p-2)]=p-2; tab[slot(b,p-1)]=p-1; }
   it[k]=iters; }
  /* waves of 64 lanes, one value each: max vs mean; and 4 values per lane (static stride) */
  for(int w=0;w<4;w++){uint32_t mx=0;double mean=0;for(int l=0;l<64;l++){uint32_t x=it[w*64+l];mean+=x;if(x>mx)mx=x;} summax+=mx;summean+=mean/64;}
  {uint32_t mx=0;double mean=0;for(int l=0;l<64;l++){uint32_t x=it[l]+it[64+l]+it[128+l]+it[192+l];mean+=x;if(x>mx)mx=x;} sum4max+=mx;sum4mean+=mean/64;}
 }
 printf("kind %d n %u: wave max/mean (1 value per lane) %.3f   (4 values per lane) %.3f   mean iters/value %.0f\n",kind,n,summax/summean,sum4max/sum4mean,summean/(count/64.0));
}
