// CPU model of the round-3 fast compressor's walks (design tool, not product code): candidates as
// the kernel picks them (two slots by 64-position group parity, the more recent 4-byte match), rows
// of 16 positions per lane, 1 KiB super-chunks, the first walk from every row start and the
// resynchronisation rounds; counts the SIMT iterations and the match lengths each phase computes.
// Build: gcc -O2 -w -o /tmp/rs tools/sc_resync_model.c     Run: /tmp/rs file...
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint32_t ld32(const uint8_t* p){uint32_t v;memcpy(&v,p,4);return v;}
static uint32_t T[8192], T2[8192], cand[65536];
static long spec_lens, spec_iters;
static int OV, FIRST;
static long n_sc, walk_iters1, rs_rounds, rs_iters, rs_lenlanes, rs_lanes_chg, first_lens, rs_lens, rs_rounds_needlen;
static int lenAt(const uint8_t* d, uint32_t q, uint32_t sce, uint32_t* enc){
  uint32_t c=cand[q]; uint32_t l=0; while(l<16 && d[c+l]==d[q+l]) ++l;
  uint32_t av=sce-q; *enc = (l==16 && av>16)?17:(l<av?l:av); return 0;}
int main(int argc,char**argv){
  if(getenv("OV")) OV=atoi(getenv("OV"));
  if(getenv("FIRST")) FIRST=atoi(getenv("FIRST"));  // the first walk from row position FIRST (lane 0: 0)
  for(int f=1;f<argc;++f){FILE*fp=fopen(argv[f],"rb");fseek(fp,0,SEEK_END);long sz=ftell(fp);fseek(fp,0,SEEK_SET);
  uint8_t*d=calloc(sz+64,1);if(fread(d,1,sz,fp)!=(size_t)sz) return 2;fclose(fp);
  for(long o=0;o<sz;o+=65536){uint32_t n=sz-o<65536?sz-o:65536; const uint8_t*b=d+o;
    memset(T,0,sizeof T);memset(T2,0,sizeof T2);
    static uint8_t match[65536];
    for(uint32_t q=0;q<n;++q){ match[q]=0; if(q+4>n) continue; uint32_t h=(ld32(b+q)*0x1e35a7bdu)>>19;
      uint32_t cls=(q>>6)&1; uint32_t*Ta=cls?T2:T,*Tb=cls?T:T2; uint32_t a=Ta[h],bb=Tb[h];
      uint32_t c1=a>bb?a:bb,c2=a>bb?bb:a; Ta[h]=q+1;
      uint32_t sce=(q/1024+1)*1024; if(sce>n) sce=n;
      int ok1=q+4<=sce && c1 && c1-1<q, ok2=q+4<=sce && c2 && c2-1<q;
      if(ok1 && ld32(b+c1-1)==ld32(b+q)){match[q]=1;cand[q]=c1-1;} else if(ok2 && ld32(b+c2-1)==ld32(b+q)){match[q]=1;cand[q]=c2-1;}
    }
    for(uint32_t sc0=0;sc0<n;sc0+=1024){ uint32_t sce=sc0+1024<n?sc0+1024:n; n_sc++;
      uint32_t S[64],E[64],P[64],mask[64];
      for(int l=0;l<64;++l){uint32_t c0=sc0+16*l;mask[l]=0;for(int i=0;i<16;++i) if(c0+i<sce && match[c0+i]) mask[l]|=1u<<i;}
      // walk: returns steps (length computations) and path/end
      #define WALK(l,sr,stop,path,mpos,pend,steps) { uint32_t c0=sc0+16*(l), ce=c0<sce?(c0+16<sce?c0+16:sce):c0; \
        uint32_t m0=(sr)<16?mask[l]>>(sr):0; uint32_t i=m0?(sr)+__builtin_ctz(m0):16; path=0; mpos=16; steps=0; uint32_t last=16,lastL=0; \
        while(i<16){ if(((stop)>>i)&1){mpos=i;break;} path|=1u<<i; last=i; uint32_t enc; lenAt(b,c0+i,sce,&enc); steps++; lastL=enc; \
          uint32_t t=i+(enc<16?enc:16); uint32_t m=mask[l]>>t; i=m?t+__builtin_ctz(m):16; } \
        pend=ce; if(last<16){uint32_t L=lastL; if(last+(L<16?L:16)>=16){ if(L==17){uint32_t q=c0+last,c=cand[q];L=16;uint32_t cap=sce-q<255?sce-q:255;while(L<cap&&b[c+L]==b[q+L])++L;} pend=c0+last+L;}} }
      int mx=0, mx0=0;
      for(int l=0;l<64;++l){uint32_t c0=sc0+16*l; uint32_t mp,st; uint32_t s0=c0+(l?FIRST:0), st0=0;
        if(OV && l>0 && c0<sce){  // speculative entry: walk the previous row from OV bytes before
          uint32_t pr=l-1, pc0=sc0+16*pr; uint32_t i=16-OV; uint32_t m0=mask[pr]>>i; i=m0?i+__builtin_ctz(m0):16;
          uint32_t pos=pc0+i;
          while(i<16){ uint32_t enc; lenAt(b,pc0+i,sce,&enc); st0++; uint32_t L=enc;
            if(L==17){uint32_t q=pc0+i,c=cand[q];L=16;uint32_t cap=sce-q<255?sce-q:255;while(L<cap&&b[c+L]==b[q+L])++L;}
            uint32_t t=i+L; if(t>=16){pos=pc0+t;break;} uint32_t m=mask[pr]>>t; i=m?t+__builtin_ctz(m):16; pos=pc0+i; }
          if(pos<c0) pos=c0;
          s0=pos; }
        spec_lens+=st0; if((int)st0>mx0) mx0=st0;
        S[l]=s0;
        if(s0<(c0+16<sce?c0+16:sce)){WALK(l,s0-c0,0,P[l],mp,E[l],st);} else {P[l]=0;E[l]=s0;st=0;}
        first_lens+=st; if((int)st>mx)mx=st;}
      walk_iters1+=mx; spec_iters+=mx0;
      for(;;){ uint32_t sn[64]; int chg=0; for(int l=0;l<64;++l){sn[l]=l?E[l-1]:sc0; if(sn[l]!=S[l]) chg++;}
        if(!chg) break; rs_rounds++; rs_lanes_chg+=chg; int mxs=0,nl=0;
        uint32_t NE[64];
        for(int l=0;l<64;++l){ NE[l]=E[l]; if(sn[l]==S[l]) continue; uint32_t c0=sc0+16*l, ce=c0<sce?(c0+16<sce?c0+16:sce):c0;
          S[l]=sn[l]; if(sn[l]>=ce){P[l]=0;NE[l]=sn[l];continue;}
          uint32_t nP,mp,ne,st; WALK(l,sn[l]-c0,P[l],nP,mp,ne,st); rs_lens+=st; if(st){nl++;} if((int)st>mxs)mxs=st;
          if(mp==16){P[l]=nP;NE[l]=ne;} else {P[l]=nP|(P[l]&~((1u<<mp)-1));} }
        for(int l=0;l<64;++l) E[l]=NE[l];
        rs_iters+=mxs; rs_lenlanes+=nl; if(nl) rs_rounds_needlen++;
      }
    }
  }}
  printf("speculative entry (OV=%d): SIMT iterations %.2f/sc, lengths %.1f/sc\n", OV, (double)spec_iters/n_sc, (double)spec_lens/n_sc);
  printf("super-chunks %ld\nfirst walk: SIMT iterations %.2f, lengths/sc %.1f\nresync: rounds %.2f/sc, rounds needing lengths %.2f, SIMT len-iterations %.2f/sc, lanes changed %.1f/sc, lanes computing %.1f/sc, lengths %.1f/sc\n",
    n_sc,(double)walk_iters1/n_sc,(double)first_lens/n_sc,(double)rs_rounds/n_sc,(double)rs_rounds_needlen/n_sc,(double)rs_iters/n_sc,(double)rs_lanes_chg/n_sc,(double)rs_lenlanes/n_sc,(double)rs_lens/n_sc);
}
