// Stochastic local search (r04) for a pair form of the stencil rule: NF
// "feature" gates over the pair's H3 bits (bs, bc, es, ec; computed once per pair)
// and NT test gates per row over the features, a0, a1, alive and (RAW = 1) the raw
// pair bits, for alive && b + e + A == 3 (rule 0, B/S2) or B3/S23 (rule 1).  Cost
// per plane and row: NF / 2 + NT; a test that reads raw pair bits needs them kept
// until the pair's second row (life_stencil.h keeps only the lower row's H3).
//   gcc -O3 -march=native -o /tmp/rsf tools/rule_search_pair_feat.c -lm
//   /tmp/rsf NF NT SEED ITERS RULE [RAW]      e.g. /tmp/rsf 3 3 2 400000 0 1
// Found for B/S2: NF = 3, NT = 3 with ec as the only raw bit (life_stencil.h
// ref_from_pair; 4.5 per row against the binary pair sum's 2 + 3).
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <math.h>
typedef unsigned __int128 u128;
typedef uint64_t u64;
static u128 var[7], f;
static int NF, NT, RAW;
#define MAXG 10
typedef struct { int in[MAXG][3]; int lut[MAXG]; } Net;
static u128 lut3(int L, u128 a, u128 b, u128 c){ u128 r=0; for(int p=0;p<8;p++) if(L>>p&1) r|=((p&4)?a:~a)&((p&2)?b:~b)&((p&1)?c:~c); return r; }
static unsigned long long rs; static unsigned rnd(){ rs^=rs<<13; rs^=rs>>7; rs^=rs<<17; return (unsigned)rs; }
static int pick(int g){ // signal ids: 0..6 inputs, 7.. gates
  if(g<NF){ int lim=4+g; int v=rnd()%lim; return v<4? v : 7+(v-4); }
  // test gate: features (7..7+NF-1), a0,a1,al (4,5,6), earlier test gates, raw (0..3) if RAW
  int n = NF + 3 + (g-NF) + (RAW?4:0); int v=rnd()%n;
  if(v<NF) return 7+v; v-=NF; if(v<3) return 4+v; v-=3; if(v<g-NF) return 7+NF+v; v-=(g-NF); return v; }
static int pc128(u128 x){ return __builtin_popcountll((u64)x)+__builtin_popcountll((u64)(x>>64)); }
static int cost(Net* n, int* bl){ int NG=NF+NT; u128 sig[7+MAXG]; for(int i=0;i<7;i++) sig[i]=var[i];
  for(int g=0; g<NG-1; g++) sig[7+g]=lut3(n->lut[g], sig[n->in[g][0]], sig[n->in[g][1]], sig[n->in[g][2]]);
  int g=NG-1; u128 a=sig[n->in[g][0]], b=sig[n->in[g][1]], c=sig[n->in[g][2]]; int err=0,L=0;
  for(int p=0;p<8;p++){ u128 m=((p&4)?a:~a)&((p&2)?b:~b)&((p&1)?c:~c); int on=pc128(f&m), off=pc128(m&~f); if(on>off){L|=1<<p; err+=off;} else err+=on; }
  if(bl)*bl=L; return err; }
int main(int argc,char**argv){
  NF=atoi(argv[1]); NT=atoi(argv[2]); rs=strtoull(argv[3],0,10)*2654435761ull+1; long iters=atol(argv[4]); int rule=atoi(argv[5]); RAW=argc>6?atoi(argv[6]):1;
  for(int i=0;i<128;i++){ int bs=i&1,bc=i>>1&1,es=i>>2&1,ec=i>>3&1,a0=i>>4&1,a1=i>>5&1,al=i>>6&1;
    int T=bs+2*bc+es+2*ec+a0+2*a1; int y= rule==0 ? (al && T==3) : (T==3 || (al && T==4)); if(y) f|=((u128)1)<<i; }
  for(int v=0;v<7;v++){ u128 m=0; for(int i=0;i<128;i++) if(i>>v&1) m|=((u128)1)<<i; var[v]=m; }
  int NG=NF+NT; int best=1000;
  for(long r=0;;r++){ Net n; for(int g=0;g<NG;g++){ for(int k=0;k<3;k++) n.in[g][k]=pick(g); n.lut[g]=rnd()&255; }
    int c=cost(&n,0); double T=2.0;
    for(long it=0; it<iters; it++){ Net m=n; int g=rnd()%NG; int w=rnd()%4;
      if(w<3) m.in[g][w]=pick(g); else m.lut[g]^=1<<(rnd()%8); if(rnd()%8==0) m.lut[g]=rnd()&255;
      int c2=cost(&m,0); if(c2<=c || exp((c-c2)/T) > (rnd()%100000)/100000.0){n=m;c=c2;} T*=0.999995; if(T<0.05)T=0.05;
      if(c==0){ int L; cost(&n,&L); printf("FOUND NF=%d NT=%d:",NF,NT); for(int k=0;k<NG;k++) printf(" g%d=L%02x(%d,%d,%d)",k,k==NG-1?L:n.lut[k],n.in[k][0],n.in[k][1],n.in[k][2]); printf("\n"); fflush(stdout); return 0; } }
    if(c<best){best=c; fprintf(stderr,"r %ld best %d\n",r,c);} } }
