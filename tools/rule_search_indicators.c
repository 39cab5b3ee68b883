// Dev: exhaustive bitop3-network search for B3/S23 over symmetric indicators.
// Build: gcc -O2 -include stdlib.h -o /tmp/rsi tools/rule_search_indicators.c && /tmp/rsi 2
// Conway next = (T==3)|(al&T==4), T = S + 2C, S,C in 0..3 popcounts of 3 planes.
// Inputs: s0 = S&1 (xor3), sY = symmetric indicator of S (1 op), cA, cB symmetric
// indicators of C (1 op each), al.  Search a k-op tail (k=2,3) over those 5 signals.
#include <stdio.h>
#include <stdint.h>
static uint32_t lut3(uint32_t a, uint32_t b, uint32_t c, int L){
  uint32_t r=0; for(int i=0;i<8;i++) if(L>>i&1){ uint32_t t=((i&4)?a:~a)&((i&2)?b:~b)&((i&1)?c:~c); r|=t;} return r;}
static int isfunc(uint32_t F, uint32_t a, uint32_t b, uint32_t c){
  int tab[8]; for(int i=0;i<8;i++)tab[i]=-1;
  for(int x=0;x<32;x++){ int idx=((a>>x&1)<<2)|((b>>x&1)<<1)|(c>>x&1); int v=F>>x&1; if(tab[idx]<0)tab[idx]=v; else if(tab[idx]!=v) return 0;}
  return 1;}
int main(int argc, char** argv){
  int k = argc>1 ? atoi(argv[1]) : 2;
  // entry x = S + 4*C + 16*al
  uint32_t F=0, s0=0, al=0; uint32_t Sind[16]={0}, Cind[16]={0};
  for(int x=0;x<32;x++){ int S=x&3, C=(x>>2)&3, a=x>>4; int T=S+2*C;
    if(T==3||(a&&T==4)) F|=1u<<x; if(S&1) s0|=1u<<x; if(a) al|=1u<<x;
    for(int m=0;m<16;m++){ if(m>>S&1) Sind[m]|=1u<<x; if(m>>C&1) Cind[m]|=1u<<x; } }
  int nfound=0;
  for(int sy=0;sy<16;sy++) for(int ca=0;ca<16;ca++) for(int cb=ca;cb<16;cb++){
    uint32_t sig[8]={s0, Sind[sy], Cind[ca], Cind[cb], al};
    int n=5;
    if(k==2){
      for(int a=0;a<n;a++)for(int b=a+1;b<n;b++)for(int c=b+1;c<n;c++)for(int L=0;L<256;L++){
        sig[5]=lut3(sig[a],sig[b],sig[c],L);
        for(int a2=0;a2<6;a2++)for(int b2=a2+1;b2<6;b2++)for(int c2=b2+1;c2<6;c2++)
          if(isfunc(F,sig[a2],sig[b2],sig[c2])){
            if(nfound<10) printf("2-op: sY=%x cA=%x cB=%x op1(%d,%d,%d,0x%02x) op2(%d,%d,%d)\n",sy,ca,cb,a,b,c,L,a2,b2,c2);
            nfound++; goto next; }
      }
    }
    next:;
  }
  printf("k=%d found %d\n",k,nfound);
  // 1-op tail: directly
  int n1=0;
  for(int sy=0;sy<16;sy++) for(int ca=0;ca<16;ca++) for(int cb=ca;cb<16;cb++){
    uint32_t sig[5]={s0, Sind[sy], Cind[ca], Cind[cb], al};
    for(int a=0;a<5;a++)for(int b=a+1;b<5;b++)for(int c=b+1;c<5;c++) if(isfunc(F,sig[a],sig[b],sig[c])) {n1++; if(n1<5) printf("1-op: sY=%x cA=%x cB=%x (%d,%d,%d)\n",sy,ca,cb,a,b,c);}
  }
  printf("1-op tails: %d\n",n1);
  return 0;
}
