// Exhaustive search (r04): every network of 4 three-input v_bitop3 gates over the
// inputs of a pair-sum row test -- q0, q1, q2 (P = H3(r-1) + H3(r), 0..6), a0, a1
// (the third row's H3, 0..3) and the cell -- for B3/S23: T = P + A == 3, or
// alive && T == 4 (P = 7 never occurs: don't care).  Gate outputs that equal an
// input or an earlier gate up to complement are skipped; threads split gate 1.
//   gcc -O3 -march=native -pthread -o /tmp/rsp tools/rule_search_pair.c
//   /tmp/rsp 1 8     (rule 1 = B3/S23, 8 threads; rule 0 = B/S2 as a check: found)
// Result: B/S2 has 3-gate networks (the kernel's ref_from_pair); B3/S23 has none
// with 4 gates (and none with 3).  5-gate ones exist (rule_search_pair_sls.c);
// the shipped form reduces the pair to other features (rule_search_pair_feat.c).
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <pthread.h>
typedef uint64_t u64;
static u64 var[6], f, care;
static int ng1; static u64 G1[6000]; static int G1d[6000][4];
static u64 lut3(int L, u64 a, u64 b, u64 c){ u64 r=0; for(int p=0;p<8;p++) if(L>>p&1) r|=((p&4)?a:~a)&((p&2)?b:~b)&((p&1)?c:~c); return r; }
static inline int consistent(u64 a, u64 b, u64 c){
  for(int p=0;p<8;p++){ u64 m=((p&4)?a:~a)&((p&2)?b:~b)&((p&1)?c:~c)&care; u64 on=f&m; if(on && on!=m) return 0; }
  return 1; }
static inline u64 canon(u64 x){ x&=care; if(x&1) x=~x&care; return x; } // row 0 is in care (q=0)
static int trivial(u64 x, u64* sig, int n){ x=canon(x); if(x==0) return 1; for(int i=0;i<n;i++) if(canon(sig[i])==x) return 1; return 0; }
static volatile int found=0; static pthread_mutex_t mu=PTHREAD_MUTEX_INITIALIZER;
static int nthreads=8;
static void* work(void* arg){
  long tid=(long)arg; u64 sig[9];
  for(int v=0;v<6;v++) sig[v]=var[v];
  for(int a=tid;a<ng1 && !found;a+=nthreads){
    sig[6]=G1[a];
    for(int i2=0;i2<7;i2++)for(int j2=i2+1;j2<7;j2++)for(int k2=j2+1;k2<7;k2++){
      for(int L2=0;L2<256;L2++){
        u64 g2=lut3(L2,sig[i2],sig[j2],sig[k2]);
        if(trivial(g2,sig,7)) continue;
        // canonical LUT choice: skip complemented duplicates (row0 output 1)
        if(g2&1) continue;
        sig[7]=g2;
        for(int i3=0;i3<8;i3++)for(int j3=i3+1;j3<8;j3++)for(int k3=j3+1;k3<8;k3++){
          if(k3<6) { /* g3 over base only: allowed */ }
          for(int L3=0;L3<256;L3++){
            u64 g3=lut3(L3,sig[i3],sig[j3],sig[k3]);
            if(g3&1) continue;
            if(trivial(g3,sig,8)) continue;
            for(int x=0;x<8;x++)for(int y=x+1;y<8;y++){
              if(consistent(g3,sig[x],sig[y])){
                pthread_mutex_lock(&mu);
                if(found<10){ printf("FOUND g1=L%02x(%d,%d,%d) g2=L%02x(%d,%d,%d) g3=L%02x(%d,%d,%d) final(g3,%d,%d)\n",
                  G1d[a][0],G1d[a][1],G1d[a][2],G1d[a][3],L2,i2,j2,k2,L3,i3,j3,k3,x,y); fflush(stdout);} found++;
                pthread_mutex_unlock(&mu);
              } } } } } }
    if(tid==0){ fprintf(stderr,"g1 %d/%d\n",a,ng1); }
  }
  return 0; }
int main(int argc,char**argv){
  int rule = argc>1?atoi(argv[1]):1;
  for(int i=0;i<64;i++){ int q0=i&1,q1=i>>1&1,q2=i>>2&1,a0=i>>3&1,a1=i>>4&1,al=i>>5&1;
    int P=q0+2*q1+4*q2, A=a0+2*a1, T=P+A; if(P==7) continue; care|=1ull<<i;
    int y = rule==0 ? (al && T==3) : (T==3 || (al && T==4)); if(y) f|=1ull<<i; }
  for(int v=0;v<6;v++){ u64 m=0; for(int i=0;i<64;i++) if(i>>v&1) m|=1ull<<i; var[v]=m; }
  // distinct gate-1 functions (canonical, non-trivial)
  u64 seen[6000]; int ns=0;
  for(int i=0;i<6;i++)for(int j=i+1;j<6;j++)for(int k=j+1;k<6;k++)for(int L=0;L<256;L++){
    u64 g=lut3(L,var[i],var[j],var[k]); if(trivial(g,var,6)) continue; u64 c=canon(g); int dup=0;
    for(int s=0;s<ns;s++) if(seen[s]==c){dup=1;break;} if(dup) continue; seen[ns++]=c;
    G1[ng1]=g; G1d[ng1][0]=L;G1d[ng1][1]=i;G1d[ng1][2]=j;G1d[ng1][3]=k; ng1++; }
  fprintf(stderr,"distinct g1: %d\n",ng1);
  if(argc>2) nthreads=atoi(argv[2]);
  pthread_t th[64]; for(long t=0;t<nthreads;t++) pthread_create(&th[t],0,work,(void*)t);
  for(int t=0;t<nthreads;t++) pthread_join(th[t],0);
  printf("solutions (up to early stop): %d\n",found);
  return 0; }
