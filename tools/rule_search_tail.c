// Dev: exhaustive bitop3-network searches for the B3/S23 rule tail.
// Build: gcc -O2 -include stdlib.h -o /tmp/rs tools/rule_search_tail.c && /tmp/rs
// exhaustive: 3 bitop3 ops over 5 inputs (s0,k0,p,mj,al) computing Conway next
#include <stdio.h>
#include <stdint.h>
static uint32_t lut3(uint32_t a, uint32_t b, uint32_t c, int L){
  uint32_t r=0; for(int i=0;i<8;i++) if(L>>i&1){ uint32_t t=((i&4)?a:~a)&((i&2)?b:~b)&((i&1)?c:~c); r|=t;} return r;}
int main(){
  uint32_t in[5]={0}; uint32_t f=0, fref=0;
  for(int x=0;x<32;x++){ int s0=x&1,k0=x>>1&1,p=x>>2&1,mj=x>>3&1,al=x>>4&1;
    for(int v=0;v<5;v++) if(x>>v&1) in[v]|=1u<<x;
    int T=s0+2*(p+k0)+4*mj; int nx=(T==3)||(al&&T==4); if(nx) f|=1u<<x; if(al&&T==3) fref|=1u<<x; }
  // note: not all (s0,k0,p,mj) combos are reachable; treat unreachable as don't care
  uint32_t care=0;
  for(int x=0;x<32;x++){ int s0=x&1,k0=x>>1&1,p=x>>2&1,mj=x>>3&1; (void)s0;
    // k0 = maj(as,bs,es), s0 = xor3: reachable pairs: (s0,k0) any of 4 (sums 0..3 -> 00,10,01,11) ok
    // p = xor3(c), mj = maj(c): any of 4. so all reachable
    care|=1u<<x; }
  for(int target=0;target<2;target++){
   uint32_t F = target? fref : f;
   int found=0;
   uint32_t sig[8]; for(int i=0;i<5;i++) sig[i]=in[i];
   for(int a1=0;a1<5&&!found;a1++)for(int b1=a1+1;b1<5;b1++)for(int c1=b1+1;c1<5;c1++)for(int L1=0;L1<256;L1++){
     sig[5]=lut3(sig[a1],sig[b1],sig[c1],L1);
     for(int a2=0;a2<6;a2++)for(int b2=a2+1;b2<6;b2++)for(int c2=b2+1;c2<6;c2++){

       for(int L2=0;L2<256;L2++){
       sig[6]=lut3(sig[a2],sig[b2],sig[c2],L2);
       for(int a3=0;a3<7;a3++)for(int b3=a3+1;b3<7;b3++)for(int c3=b3+1;c3<7;c3++){
         // is F a function of sig[a3],sig[b3],sig[c3]?
         int tab[8]; for(int i=0;i<8;i++)tab[i]=-1; int ok=1;
         for(int x=0;x<32&&ok;x++){ if(!(care>>x&1))continue; int idx=((sig[a3]>>x&1)<<2)|((sig[b3]>>x&1)<<1)|(sig[c3]>>x&1); int v=F>>x&1; if(tab[idx]<0)tab[idx]=v; else if(tab[idx]!=v) ok=0;}
         if(ok){ printf("target %d found: op1(%d,%d,%d,0x%02x) op2(%d,%d,%d,0x%02x) op3(%d,%d,%d)\n",target,a1,b1,c1,L1,a2,b2,c2,L2,a3,b3,c3); found=1; goto done;}
       }}}
   }
   done: if(!found) printf("target %d: no 3-op network (op2 using op1)\n",target);
  }
  return 0;
}
