// Stochastic local search (r04) for v_bitop3 networks of NG gates over the
// pair-sum row test's inputs q0, q1, q2, a0, a1, alive (see rule_search_pair.c):
// B3/S23, T = P + A == 3 or alive && T == 4.  The final gate's truth table is
// fitted; the others mutate under annealing, with restarts.  NQ > 0 restricts the
// first NQ gates to the pair alone (shared by the pair's two rows).
//   gcc -O3 -march=native -o /tmp/sls tools/rule_search_pair_sls.c -lm
//   /tmp/sls NG SEED ITERS [NQ]      e.g. /tmp/sls 5 11 400000
// Found: 5-gate networks with NQ = 0 and NQ = 1 (r04's first B3/S23 pair form,
// 5 gates per row on the binary pair sum; since superseded by the 4 features +
// 4 gates of rule_search_pair_feat.c, life_stencil.h conway_from_pair).
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <math.h>
typedef uint64_t u64;
static u64 var[6], f, care;
#define MAXG 8
static int NG, NQ;
typedef struct { int in[MAXG][3]; int lut[MAXG]; } Net;
static u64 lut3(int L, u64 a, u64 b, u64 c){ u64 r=0; for(int p=0;p<8;p++) if(L>>p&1) r|=((p&4)?a:~a)&((p&2)?b:~b)&((p&1)?c:~c); return r; }
static int cost(Net* n, int* bestlut){
  u64 sig[6+MAXG]; for(int i=0;i<6;i++) sig[i]=var[i];
  for(int g=0; g<NG-1; g++) sig[6+g]=lut3(n->lut[g], sig[n->in[g][0]], sig[n->in[g][1]], sig[n->in[g][2]]);
  int g=NG-1; u64 a=sig[n->in[g][0]], b=sig[n->in[g][1]], c=sig[n->in[g][2]];
  int err=0, L=0;
  for(int p=0;p<8;p++){ u64 m=((p&4)?a:~a)&((p&2)?b:~b)&((p&1)?c:~c)&care; int on=__builtin_popcountll(f&m), off=__builtin_popcountll(m&~f);
    if(on>off){ L|=1<<p; err+=off; } else err+=on; }
  if(bestlut) *bestlut=L; return err; }
static unsigned long long rs;
static unsigned rnd(){ rs^=rs<<13; rs^=rs>>7; rs^=rs<<17; return (unsigned)rs; }
static int pick(int g){ if(g<NQ){ int lim=3+g; int v=rnd()%lim; return v<3? v : 6+(v-3); } return rnd()%(6+g); }
static void randgate(Net* n, int g){ for(int k=0;k<3;k++) n->in[g][k]=pick(g); n->lut[g]=rnd()&255; }
int main(int argc,char**argv){
  NG=atoi(argv[1]); NQ=argc>4?atoi(argv[4]):0; rs=strtoull(argv[2],0,10)*2654435761ull+1; long iters=atol(argv[3]);
  for(int i=0;i<64;i++){ int q0=i&1,q1=i>>1&1,q2=i>>2&1,a0=i>>3&1,a1=i>>4&1,al=i>>5&1;
    int P=q0+2*q1+4*q2, A=a0+2*a1, T=P+A; if(P==7) continue; care|=1ull<<i; if(T==3||(al&&T==4)) f|=1ull<<i; }
  for(int v=0;v<6;v++){ u64 m=0; for(int i=0;i<64;i++) if(i>>v&1) m|=1ull<<i; var[v]=m; }
  int best_overall=1000;
  for(long restart=0; ; restart++){
    Net n; for(int g=0;g<NG;g++) randgate(&n,g);
    // final gate should use the previous gate
    int c=cost(&n,0); double T=2.0;
    for(long it=0; it<iters; it++){
      Net m=n; int g=rnd()%NG; int what=rnd()%4;
      if(what<3){ m.in[g][what]=pick(g); } else if(g<NG-1) m.lut[g]^=1<<(rnd()%8); else m.in[g][rnd()%3]=pick(g);
      if(g<NG-1 && rnd()%8==0) m.lut[g]=rnd()&255;
      int c2=cost(&m,0);
      if(c2<=c || exp((c-c2)/T) > (rnd()%100000)/100000.0){ n=m; c=c2; }
      T*=0.999995; if(T<0.05) T=0.05;
      if(c==0){ int L; cost(&n,&L); printf("FOUND NG=%d:", NG); for(int k=0;k<NG;k++) printf(" g%d=L%02x(%d,%d,%d)", k, k==NG-1?L:n.lut[k], n.in[k][0],n.in[k][1],n.in[k][2]); printf("\n"); fflush(stdout); return 0; }
    }
    if(c<best_overall){ best_overall=c; fprintf(stderr,"restart %ld best err %d\n", restart, c); }
  }
}
